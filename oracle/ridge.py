"""Oracle: ridge picking and bootstrap resampling in float64 numpy (TEST INFRASTRUCTURE ONLY).

Follows, function by function:
  extract_ridge_ref_idx   modules/utils.py:621-678
  bootstrap_disp          apis/imaging_classes.py:8-48  (VSG stack of random.sample(range(1, n), k)
                          windows -> compute_disp_image(end_x=0, start_x=-150) -> ridge per mode)
Pinned by tests/golden/ridge.npz (the reference run in the survey container, make_golden.py).
"""
from __future__ import annotations

import random

import numpy as np
import scipy.signal

from . import disp as odisp
from . import vsg as ovsg


def extract_ridge_ref_idx(freq, vel, fv_map, ref_freq_idx=None, sigma=25, vel_max=400, ref_vel=None,
                          return_picks=False):
    """modules/utils.py:621-678: vel ascending (reversed to the map's row order), fv_map [Nvel, Nfreq].
    return_picks=True also returns the raw picks before savgol (the walk's per-column argmax)."""
    vel = vel[::-1]
    if ref_freq_idx is None:
        max_idx = np.abs(vel_max - vel).argmin()
        return vel[max_idx:][np.argmax(fv_map[max_idx:], axis=0)]
    out = np.zeros(len(freq))
    if ref_vel is None:
        out[ref_freq_idx] = vel[np.argmax(fv_map[:, ref_freq_idx])]
        for i in list(range(ref_freq_idx - 1, -1, -1)) + list(range(ref_freq_idx + 1, len(freq))):
            prev = out[i + 1] if i < ref_freq_idx else out[i - 1]
            mask = (vel > prev - sigma) & (vel < prev + sigma)
            out[i] = vel[mask][np.argmax(fv_map[mask, i])]
    else:
        vr = ref_vel(freq)
        for i in range(len(freq)):
            mask = (vel > vr[i] - sigma) & (vel < vr[i] + sigma)
            out[i] = vel[mask][np.argmax(fv_map[mask, i])]
    sm = scipy.signal.savgol_filter(out, 25, 2)
    return (sm, out) if return_picks else sm


def bootstrap_disp(wins, bt_size, bt_times, sigma, pivot, start_x, end_x, ref_freq_idx, freq_lb, freq_up, ref_vel,
                   rand=random):
    """apis/imaging_classes.py:8-48 on oracle windows (dicts of data, x_axis, t_axis, veh_state_x/_t)."""
    ridge = [[] for _ in freq_lb]
    freqs = None
    cache = {}
    for _ in range(bt_times):
        sel = rand.sample(range(1, len(wins)), bt_size)
        gs = []
        for i in sel:
            if i not in cache:
                cache[i] = ovsg.virtual_shot_gather(wins[i], include_other_side=True, norm=False, pivot=pivot,
                                                    start_x=start_x, end_x=end_x, wlen=2)
            gs.append(cache[i])
        xcf = ovsg.stack([g[0] for g in gs])
        gx, gt = gs[0][1], gs[0][2]
        fv = odisp.compute_disp_image(xcf, gx, gt, start_x=-150, end_x=0)
        freqs = np.arange(0.8, 25, 0.1)
        vels = np.arange(200, 1200)
        for m in range(len(freq_lb)):
            band = (freqs >= freq_lb[m]) & (freqs < freq_up[m])
            ridge[m].append(extract_ridge_ref_idx(freqs[band], vels, fv[:, band],
                                                  ref_freq_idx=ref_freq_idx[m] - int(np.sum(freqs < freq_lb[m])),
                                                  sigma=sigma[m], vel_max=800, ref_vel=ref_vel[m]))
    return ridge, freqs
