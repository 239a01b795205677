"""Oracle: restatement of the dispersion (f-v) transform in float64 numpy (TEST INFRASTRUCTURE ONLY).

Follows:
  fk      modules/utils.py:236-248   |fftshift(fft2(data, s=[nk, nf]))| and its axes
  map_fv  modules/utils.py:457-475   optional per-trace L1 norm; interp2d(fft_k, fft_f, FK.T) linear
                                     (bilinear, queries sorted, clamped to the grid), float32 map,
                                     savgol_filter(25, 4, axis=0, mode='interp'), transpose
  VirtualShotGather.compute_disp_image  apis/virtual_shot_gather.py:247-258
  SurfaceWaveDispersion._naive_disp     apis/dispersion_classes.py:24-32
The bilinear evaluation is written out explicitly (FITPACK fpbisp's interval search with the
argument clamped to [t_b, t_e]); the Savitzky-Golay step calls scipy.signal.savgol_filter, which is
the reference's own third-party call.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.signal


def fk(data, dx, dt):
    nch, nt = np.shape(data)
    nf = 2 ** (1 + math.ceil(math.log(nt, 2)))
    nk = 2 ** (1 + math.ceil(math.log(nch, 2)))
    fft_f = np.arange(-nf / 2, nf / 2) / nf / dt
    fft_k = np.arange(-nk / 2, nk / 2) / nk / dx
    res = np.abs(np.fft.fftshift(np.fft.fft2(data, s=[nk, nf])))
    return res, fft_f, fft_k


def _interval(grid, q):
    """fpbisp: clamp to [grid[0], grid[-1]], then l with grid[l] <= q < grid[l+1] (l <= n-2)."""
    q = np.clip(q, grid[0], grid[-1])
    l = np.clip(np.searchsorted(grid, q, side="right") - 1, 0, len(grid) - 2)
    a = (q - grid[l]) / (grid[l + 1] - grid[l])
    return l, a


def bilinear(fk_res, fft_f, fft_k, kq, fq):
    """interp2d(fft_k, fft_f, fk_res.T)(kq, fq) for a scalar fq; kq sorted ascending first."""
    kq = np.sort(np.atleast_1d(kq), kind="mergesort")
    m, a = _interval(fft_k, kq)
    j, b = _interval(fft_f, np.array([fq]))
    j, b = j[0], b[0]
    z00 = fk_res[m, j]
    z10 = fk_res[m + 1, j]
    z01 = fk_res[m, j + 1]
    z11 = fk_res[m + 1, j + 1]
    return (1 - a) * (1 - b) * z00 + a * (1 - b) * z10 + (1 - a) * b * z01 + a * b * z11


def map_fv(data, dx, dt, freqs, vels, norm=False):
    if norm:
        data = data / np.linalg.norm(data, axis=-1, keepdims=True, ord=1)
    res, fft_f, fft_k = fk(data, dx, dt)
    fv = np.zeros((len(freqs), len(vels)), dtype=np.float32)
    ones = np.ones(len(vels))
    for i, fr in enumerate(freqs):
        fv[i, :] = bilinear(res, fft_f, fft_k, np.divide(ones * fr, vels), fr)
    fv = scipy.signal.savgol_filter(fv, 25, 4, axis=0)
    return fv.T


def compute_disp_image(xcf, gx, gt, freqs=None, vels=None, norm=False, start_x=None, end_x=None):
    freqs = np.arange(0.8, 25, 0.1) if freqs is None else freqs
    vels = np.arange(200, 1200) if vels is None else vels
    start_x = gx[0] if start_x is None else start_x
    end_x = gx[-1] if end_x is None else end_x
    s = np.abs(gx - start_x).argmin()
    e = np.abs(gx - end_x).argmin()
    return map_fv(xcf[s:e + 1], 8.16, gt[1] - gt[0], freqs, vels, norm)


def naive_disp(data, x_axis, t_axis, freqs, vels, start_x, end_x, norm=True):
    dist = end_x - start_x
    dx = x_axis[1] - x_axis[0]
    s = int(np.argmax(x_axis >= start_x))
    nx = int(dist / dx)
    return map_fv(data[s:s + nx], dx, t_axis[1] - t_axis[0], freqs, vels, norm)


def pick_ok(ref_fv, picks):
    """Pick contract: pick j is accepted iff ref_fv[pick_j, j] == max_v ref_fv[:, j]."""
    ref_fv = np.asarray(ref_fv)
    cols = np.arange(ref_fv.shape[1])
    return ref_fv[picks, cols] == ref_fv.max(axis=0)
