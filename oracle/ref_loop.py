"""CPU baseline with the reference's loop structure (TEST / BENCH INFRASTRUCTURE ONLY).

This is the "reference CPU path" bench.py times on the GPU box's host (cpu_baseline.kind = "port"):
the per-pass, per-row, per-sub-window ``scipy.signal.correlate(..., mode='valid', method='fft')``
calls of XCORR_vshot / XCORR_two_traces (modules/utils.py:253-314), the scipy ``interp1d`` trajectory
of preprocessing_window (apis/virtual_shot_gather.py:111-126), a Python ``sum()`` / ``len`` stack
(apis/imaging_classes.py:106-107) and map_fv with a FITPACK bilinear spline and savgol_filter
(modules/utils.py:457-475, ``interp2d`` -> ``RectBivariateSpline(kx=ky=1, s=0)``).  It is single-threaded
like the reference.  Its outputs are checked against the golden vectors in tests/test_oracle.py, so
the timed loop computes the same thing as the reference.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.interpolate
import scipy.signal


def _circ(a, b):
    """correlate(repeat1d(a), b, 'valid', 'fft'), as the reference evaluates one row."""
    return scipy.signal.correlate(np.hstack((a, a[:-1])), b, mode="valid", method="fft")


def _sub_windows(n, w, hop):
    return range(max((n - w) // hop + 1, 0))


def gather(data, x_axis, t_axis, vx, vt, pivot, start_x, end_x, wlen=2, twin=4, delta_t=1, two_sided=True):
    """One pass: VirtualShotGather(window, include_other_side=two_sided, norm=False).XCF_out."""
    f = scipy.interpolate.interp1d(vx, vt, fill_value="extrapolate")
    dt = t_axis[1] - t_axis[0]
    w = int(wlen / dt)
    hop = int(w * 0.5)
    nsamp = int(twin // dt)
    ip = int(np.argmax(x_axis >= pivot))
    i0 = int(np.argmax(x_axis >= start_x))
    i1 = int(np.abs(x_axis - end_x).argmin())
    data = data / np.linalg.norm(data)
    sides = []
    for sgn in ((1, -1) if two_sided else (1,)):
        pt = int(np.argmax(t_axis >= f(pivot) + sgn * delta_t))
        out = np.zeros((i1 - i0, w))
        for r in range(i0, i1):
            shared = r <= ip if sgn > 0 else r >= ip
            if shared:
                sl = slice(pt, pt + nsamp) if sgn > 0 else slice(pt - nsamp, pt)
            else:
                ti = int(np.argmax(t_axis >= f(x_axis[r]) + sgn * delta_t))
                sl = slice(ti, ti + nsamp) if sgn > 0 else slice(ti - nsamp, ti)
            p, q = data[ip, sl], data[r, sl]
            acc = np.zeros(w)
            nwin = (p.size - w) // hop + 1
            for s in _sub_windows(p.size, w, hop):
                a, b = p[s * hop:s * hop + w], q[s * hop:s * hop + w]
                if sgn > 0:
                    acc += _circ(a, b) if shared else _circ(b, a)
                else:
                    acc += scipy.signal.correlate(b, np.hstack((a, a[:-1])), mode="valid", method="fft") \
                        if shared else _circ(a, b)
            acc = np.roll(acc, w // 2)
            if nwin > 0:
                acc /= nwin
            out[r - i0] = acc
        with np.errstate(invalid="ignore", divide="ignore"):
            out = out / np.amax(out[ip - i0])
        sides.append(out[:, ::-1] if sgn > 0 else out)
    g = sides[0]
    if two_sided:
        with np.errstate(invalid="ignore"):
            ok = np.linalg.norm(sides[1], axis=-1) > 0
        g = g.copy()
        g[ok] = (g[ok] + sides[1][ok]) / 2
    gx = x_axis[i0:i1] - x_axis[ip]
    gt = (np.arange(w) - w // 2) * dt
    return g, gx, gt


def map_fv(data, dx, dt, freqs, vels):
    nch, nt = data.shape
    nf = 2 ** (1 + math.ceil(math.log(nt, 2)))
    nk = 2 ** (1 + math.ceil(math.log(nch, 2)))
    fft_f = np.arange(-nf / 2, nf / 2) / nf / dt
    fft_k = np.arange(-nk / 2, nk / 2) / nk / dx
    res = np.abs(np.fft.fftshift(np.fft.fft2(data, s=[nk, nf])))
    spl = scipy.interpolate.RectBivariateSpline(fft_k, fft_f, res, kx=1, ky=1, s=0)
    fv = np.zeros((len(freqs), len(vels)), dtype=np.float32)
    for i, fr in enumerate(freqs):
        kq = np.sort(np.divide(np.ones(len(vels)) * fr, vels), kind="mergesort")
        fv[i] = spl(kq, np.array([fr]))[:, 0]
    return scipy.signal.savgol_filter(fv, 25, 4, axis=0).T


def disp_image(g, gx, gt, start_x=-200, end_x=0, freqs=None, vels=None):
    freqs = np.arange(0.8, 25, 0.1) if freqs is None else freqs
    vels = np.arange(200, 1200) if vels is None else vels
    s = np.abs(gx - start_x).argmin()
    e = np.abs(gx - end_x).argmin()
    return map_fv(g[s:e + 1], 8.16, gt[1] - gt[0], freqs, vels)


def class_images(windows, slots, n_slot, pivot, start_x, end_x):
    """Per class: sum(gathers) / len, then its f-v image (call stack A of SURVEY §3)."""
    acc = [None] * n_slot
    cnt = [0] * n_slot
    gx = gt = None
    for (data, x_axis, t_axis, vx, vt), s in zip(windows, slots):
        g, gx, gt = gather(data, x_axis, t_axis, vx, vt, pivot, start_x, end_x)
        acc[s] = g if acc[s] is None else acc[s] + g
        cnt[s] += 1
    stacks = [a / c for a, c in zip(acc, cnt) if c]
    return stacks, [disp_image(st, gx, gt) for st in stacks]



def timed_worker(path, first, budget_s):
    """One single-threaded worker of the all-core CPU baseline: gathers of the windows saved in
    ``path`` (.npz: wins [n, C, T] float32, x_axis, t_axis, vx/vt [n, L], pivot, start_x, end_x -- scalars,
    or one per window for sliding-pivot units), round robin from window ``first``, until ``budget_s`` has
    elapsed.  Returns (done, seconds)."""
    import time
    z = np.load(path, allow_pickle=False)
    wins, vx, vt = z["wins"], z["vx"], z["vt"]
    x_axis, t_axis = z["x_axis"], z["t_axis"]
    n, done = wins.shape[0], 0
    piv, sx, ex = (np.broadcast_to(np.asarray(z[k], dtype=np.float64), (n,)) for k in ("pivot", "start_x", "end_x"))
    t0 = time.perf_counter()
    while True:
        i = (first + done) % n
        gather(np.asarray(wins[i], np.float64), x_axis, t_axis, vx[i], vt[i], piv[i], sx[i], ex[i])
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            return done, el


if __name__ == "__main__":  # python -m oracle.ref_loop SAMPLE.npz FIRST BUDGET_S  -> "done seconds"
    import sys
    d, t = timed_worker(sys.argv[1], int(sys.argv[2]), float(sys.argv[3]))
    print(d, t)
