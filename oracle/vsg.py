"""Oracle: restatement of the virtual-shot-gather path in float64 numpy (TEST INFRASTRUCTURE ONLY).

Follows, function by function:
  preprocessing_window          apis/virtual_shot_gather.py:111-126
  xcorr_two_traces_based_on_traj apis/virtual_shot_gather.py:14-43
  XCORR_vshot                   modules/utils.py:289-314
  XCORR_two_traces              modules/utils.py:253-270 (repeat1d 250-251)
  post_processing_XCF           apis/virtual_shot_gather.py:129-142
  construct_shot_gather[_other_side] apis/virtual_shot_gather.py:145-180
  VirtualShotGather.__init__    apis/virtual_shot_gather.py:184-192
The circular correlation ``correlate(repeat1d(a), b, 'valid')`` is evaluated as
``irfft(rfft(a) * conj(rfft(b)))`` (identical to 1e-15); the argument order of every call is kept
as in the reference so that the lag conventions come out of the arithmetic, not from a derivation.
"""
from __future__ import annotations

import numpy as np


def interp1d_extrap(xp, yp):
    """scipy.interpolate.interp1d(xp, yp, kind='linear', fill_value='extrapolate') (SciPy 1.15.3,
    ``_call_linear``): mergesort the abscissae, searchsorted(left), clip to [1, n-1], then
    ``slope * (x - x_lo) + y_lo`` with ``slope = (y_hi - y_lo) / (x_hi - x_lo)``."""
    order = np.argsort(xp, kind="mergesort")
    x = np.asarray(xp, dtype=np.float64)[order]
    y = np.asarray(yp, dtype=np.float64)[order]

    def f(xq):
        xq = np.asarray(xq, dtype=np.float64)
        i = np.clip(np.searchsorted(x, xq), 1, len(x) - 1)
        lo = i - 1
        slope = (y[i] - y[lo]) / (x[i] - x[lo])
        return slope * (xq - x[lo]) + y[lo]

    return f


def veh_state_xt(veh_state, start_x_tracking, dist_trk, t_trk):
    """SurfaceWaveWindow._preprocess_veh_state (apis/data_classes.py:34-39)."""
    veh_state = np.asarray(veh_state, dtype=np.float64)
    ok = ~np.isnan(veh_state)
    tmp = veh_state[ok].astype(int)
    i0 = np.abs(start_x_tracking - dist_trk).argmin()
    return dist_trk[np.where(ok)[0] + i0], t_trk[tmp]


def circ_xcorr(a, b):
    """correlate(repeat1d(a), b, mode='valid'): z[k] = sum_n a[(n + k) % w] * b[n]."""
    w = a.shape[-1]
    return np.fft.irfft(np.fft.rfft(a) * np.conj(np.fft.rfft(b)), n=w)


def _nwin(nt, w, hop):
    return (nt - w) // hop + 1


def xcorr_vshot(data, ivs, w, hop, reverse=False):
    """XCORR_vshot: every row shares the pivot row's time slice."""
    nch, nt = data.shape
    nwin = _nwin(nt, w, hop)
    out = np.zeros((nch, w))
    for i in range(max(nwin, 0)):
        seg = data[:, i * hop:i * hop + w]
        p = seg[ivs]
        if reverse:  # correlate(row, repeat1d(p)) = c(p, row)[w - 1 - k]
            out += circ_xcorr(p[None, :], seg)[:, ::-1]
        else:
            out += circ_xcorr(p[None, :], seg)
    if nwin == 0:
        return np.zeros((nch, w))
    return np.roll(out, w // 2, axis=-1) / nwin


def xcorr_two(tr1, tr2, w, hop):
    """XCORR_two_traces(tr1, tr2): correlate(repeat1d(tr1_window), tr2_window)."""
    nwin = _nwin(tr1.size, w, hop)
    out = np.zeros(w)
    for i in range(max(nwin, 0)):
        out += circ_xcorr(tr1[i * hop:i * hop + w], tr2[i * hop:i * hop + w])
    out = np.roll(out, w // 2)
    if nwin > 0:
        out /= nwin
    return out


def xcorr_traj(data, t_axis, pivot_idx, f, end_idx, w, w_alloc, hop, nsamp, x_axis, delta_t, reverse):
    nch = abs(end_idx - pivot_idx) - 1 + (1 if reverse else 0)
    out = np.zeros((nch, w_alloc))
    lo, hi = min(pivot_idx, end_idx), max(pivot_idx, end_idx)
    if reverse:
        lo -= 1
    for k, xi in enumerate(range(lo + 1, hi)):
        t = f(x_axis[xi])
        t = t - delta_t if reverse else t + delta_t
        ti = int(np.argmax(t_axis >= t))
        if reverse:
            piv, rcv = data[pivot_idx, ti - nsamp:ti], data[xi, ti - nsamp:ti]
            out[k] = xcorr_two(piv, rcv, w, hop)   # vs = pivot, vr = receiver
        else:
            piv, rcv = data[pivot_idx, ti:ti + nsamp], data[xi, ti:ti + nsamp]
            out[k] = xcorr_two(rcv, piv, w, hop)   # vs = receiver, vr = pivot
    return out


def _prep(win, pivot, delta_t, start_x, end_x, twin):
    f = interp1d_extrap(win["veh_state_x"], win["veh_state_t"])
    x_axis, t_axis, data = win["x_axis"], win["t_axis"], win["data"]
    dt = t_axis[1] - t_axis[0]
    pivot_idx = int(np.argmax(x_axis >= pivot))
    pt = int(np.argmax(t_axis >= f(pivot) + delta_t))
    start_idx = int(np.argmax(x_axis >= start_x))
    end_idx = int(np.abs(x_axis - end_x).argmin())
    nsamp = int(twin // dt)
    data = data / np.linalg.norm(data)
    return f, dt, pivot_idx, pt, start_idx, end_idx, nsamp, data


def _post(x_axis, pivot_idx, start_idx, end_idx, xcf, dt, norm, norm_amp, reverse):
    gx = x_axis[start_idx:end_idx] - x_axis[pivot_idx]
    nt = xcf.shape[-1]
    gt = (np.arange(nt) - nt // 2) * dt
    with np.errstate(invalid="ignore", divide="ignore"):
        if norm:
            xcf = xcf / np.linalg.norm(xcf, axis=-1, keepdims=True)
        if norm_amp:
            xcf = xcf / np.amax(xcf[pivot_idx - start_idx])
    if not reverse:
        xcf = xcf[:, ::-1]
    return xcf, gx, gt


def shot_gather(win, pivot, start_x, end_x, wlen=2, norm=True, norm_amp=True, time_window_to_xcorr=4,
                delta_t=1, other_side=False):
    sgn = -1 if other_side else 1
    f, dt, pivot_idx, pt, start_idx, end_idx, nsamp, data = _prep(win, pivot, sgn * delta_t, start_x, end_x,
                                                                   time_window_to_xcorr)
    w = int(wlen / dt)
    hop = int(w * 0.5)
    w_alloc = int(wlen // dt)
    if w_alloc != w:
        raise ValueError(f"window length mismatch: int(wlen // dt) = {w_alloc} != int(wlen / dt) = {w}")
    x_axis, t_axis = win["x_axis"], win["t_axis"]
    if not other_side:
        a = xcorr_vshot(data[start_idx:pivot_idx + 1, pt:pt + nsamp], pivot_idx - start_idx, w, hop)
        b = xcorr_traj(data, t_axis, pivot_idx, f, end_idx, w, w_alloc, hop, nsamp, x_axis, delta_t, False)
    else:
        b = xcorr_vshot(data[pivot_idx:end_idx, pt - nsamp:pt], 0, w, hop, reverse=True)
        a = xcorr_traj(data, t_axis, pivot_idx, f, start_idx, w, w_alloc, hop, nsamp, x_axis, delta_t, True)
    xcf = np.concatenate((a, b), axis=0)
    return _post(x_axis, pivot_idx, start_idx, end_idx, xcf, dt, norm, norm_amp, other_side)


def virtual_shot_gather(win, include_other_side=False, **kw):
    """VirtualShotGather.__init__ (apis/virtual_shot_gather.py:184-192) -> (XCF_out, x_axis, t_axis)."""
    xcf, gx, gt = shot_gather(win, other_side=False, **kw)
    if include_other_side:
        other, _, _ = shot_gather(win, other_side=True, **kw)
        with np.errstate(invalid="ignore"):
            ok = np.linalg.norm(other, axis=-1) > 0
        xcf = xcf.copy()
        xcf[ok] = (xcf[ok] + other[ok]) / 2
    return xcf, gx, gt


def stack(gathers):
    """sum(images) / len(images) (apis/imaging_classes.py:106-107; __add__/__truediv__ 195-210)."""
    acc = gathers[0].copy()
    for g in gathers[1:]:
        n = min(acc.shape[-1], g.shape[-1])
        acc[:, :n] += g[:, :n]
    return acc / len(gathers)


def window_from_arrays(q_or_data, x_axis, t_axis, veh_state, start_x_tracking, dist_trk, t_trk, quant=2.0 ** -12):
    data = np.asarray(q_or_data)
    if data.dtype == np.int16:
        data = data.astype(np.float64) * quant
    vx, vt = veh_state_xt(veh_state, start_x_tracking, dist_trk, t_trk)
    return dict(data=np.asarray(data, dtype=np.float64), x_axis=x_axis, t_axis=t_axis, veh_state_x=vx,
                veh_state_t=vt)
