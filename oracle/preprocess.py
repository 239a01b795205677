"""Oracle: bandpass + mutes restated in float64 numpy (TEST INFRASTRUCTURE ONLY).

Follows:
  bandpass_data   modules/utils.py:179-189 -> scipy.signal.butter(10, [flo, fhi] / fNy, 'band',
                  output='sos') then sosfiltfilt(axis=1).  sosfiltfilt (SciPy 1.15.3) is restated:
                  odd extension of padlen = 3 * (2 * n_sections + 1 - min(#zero b2, #zero a2)) samples
                  at both ends, zi = sosfilt_zi(sos) scaled by the first sample, forward sosfilt,
                  reverse, again, reverse, trim.  Pure-Python recursion: small inputs only.
  mute_along_traj apis/data_classes.py:49-72
  mute_along_time apis/data_classes.py:100-104
"""
from __future__ import annotations

import numpy as np
import scipy.signal

from oracle.vsg import interp1d_extrap


def butter_sos(dt, flo, fhi, order=10):
    fny = 0.5 / dt
    return scipy.signal.butter(order, [flo / fny, fhi / fny], analog=False, btype="band", output="sos")


def _sosfilt(sos, x, zi):
    y = np.array(x, dtype=np.float64)
    z = np.array(zi, dtype=np.float64)
    for s in range(sos.shape[0]):
        b0, b1, b2, _, a1, a2 = sos[s]
        z0, z1 = z[s]
        out = np.empty_like(y)
        for n in range(y.size):  # transposed direct form II, as scipy's _sosfilt
            xn = y[n]
            yn = b0 * xn + z0
            z0 = b1 * xn - a1 * yn + z1
            z1 = b2 * xn - a2 * yn
            out[n] = yn
        y = out
    return y


def sosfiltfilt_1d(sos, x):
    n_sec = sos.shape[0]
    padlen = 3 * (2 * n_sec + 1 - min(int((sos[:, 2] == 0).sum()), int((sos[:, 5] == 0).sum())))
    x = np.asarray(x, dtype=np.float64)
    ext = np.concatenate((2 * x[0] - x[padlen:0:-1], x, 2 * x[-1] - x[-2:-(padlen + 2):-1]))
    zi = scipy.signal.sosfilt_zi(sos)
    y = _sosfilt(sos, ext, zi * ext[0])
    y = _sosfilt(sos, y[::-1], zi * y[-1])[::-1]
    return y[padlen:-padlen]


def bandpass_data(data, dt, flo, fhi):
    sos = butter_sos(dt, flo, fhi)
    return np.stack([sosfiltfilt_1d(sos, row) for row in np.asarray(data, dtype=np.float64)])


def bandpass_data_scipy(data, dt, flo, fhi):
    """bandpass_data exactly as the reference calls it (modules/utils.py:179-189: scipy.signal.sosfiltfilt on
    axis 1, SciPy's compiled sosfilt): the CPU baseline of bench.py --workload prep (the pure-Python
    restatement above is the checker for small inputs)."""
    return scipy.signal.sosfiltfilt(butter_sos(dt, flo, fhi), data, axis=1)


def tukey(n, alpha):
    """scipy.signal.windows.tukey(n, alpha), sym=True."""
    if n <= 0:
        return np.array([])
    if n == 1:
        return np.ones(1)
    if alpha <= 0:
        return np.ones(n)
    if alpha >= 1:
        return scipy.signal.windows.hann(n)
    k = np.arange(n)
    width = int(np.floor(alpha * (n - 1) / 2.0))
    n1, n2 = k[:width + 1], k[width + 1:n - width - 1]
    n3 = k[n - width - 1:]
    w1 = 0.5 * (1 + np.cos(np.pi * (-1 + 2.0 * n1 / alpha / (n - 1))))
    w2 = np.ones(n2.shape)
    w3 = 0.5 * (1 + np.cos(np.pi * (-2.0 / alpha + 1 + 2.0 * n3 / alpha / (n - 1))))
    return np.concatenate((w1, w2, w3))


def mute_along_traj(data, x_axis, t_axis, veh_state_x, veh_state_t, offset=200, alpha=0.3, delta_x=20):
    f = interp1d_extrap(veh_state_t, veh_state_x)
    car = f(t_axis)
    dx = x_axis[1] - x_axis[0]
    nx = x_axis.size
    n_samp = int(offset / dx)
    taper = tukey(n_samp, alpha)
    out = np.array(data, dtype=np.float64)
    for k in range(t_axis.size):
        m = np.zeros(nx)
        c = int(np.argmax(x_axis > car[k] - offset / 2 + delta_x))
        s = max(0, c - n_samp // 2)
        e = min(nx, c + n_samp // 2)
        ts = s + n_samp // 2 - c
        m[s:e] = taper[ts:ts + e - s]
        out[:, k] *= m
    return out


def mute_along_time(data, alpha=0.3):
    return np.asarray(data, dtype=np.float64) * tukey(data.shape[-1], alpha)[None, :]


def find_noise_idx(data, noise_threshold=5, empty_tr=False):
    """modules/utils.py:316-321 (np.argmax of the condition: 0 when no trace qualifies)."""
    if not empty_tr:
        return np.argmax(np.max(data, axis=1) > noise_threshold)
    return np.argmax(np.linalg.norm(data, axis=1) < noise_threshold)


def impute_noisy_trace(data, noise_idx):
    """modules/utils.py:323-329 (an interior trace becomes the SUM of its neighbours)."""
    if noise_idx + 1 == data.shape[0]:
        data[noise_idx] = data[noise_idx - 1]
    elif noise_idx == 0:
        data[noise_idx] = data[noise_idx + 1]
    else:
        data[noise_idx] = (data[noise_idx - 1] + data[noise_idx + 1])


def surface_wave_prep(data, dt, method="surface_wave", flo=1.2, fhi=30, impute_noise_traces=True, noise_threshold=5,
                      impute_empty_traces=True, scipy_filter=False):
    """TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71) -> data_for_imaging.
    scipy_filter: bandpass through scipy.signal.sosfiltfilt as the reference calls it (large records)."""
    d = (bandpass_data_scipy if scipy_filter else bandpass_data)(data, dt, flo, fhi)  # the filtered copy
    if impute_empty_traces:
        impute_noisy_trace(d, find_noise_idx(d, noise_threshold=noise_threshold, empty_tr=True))
    if impute_noise_traces:
        impute_noisy_trace(d, find_noise_idx(d, noise_threshold=noise_threshold, empty_tr=False))
    if method == "surface_wave":
        d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return d
