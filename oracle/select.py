"""Oracle: surface-wave window selection restated as a plain loop (TEST INFRASTRUCTURE ONLY).

Follows SurfaceWaveSelector.locate_windows (apis/data_classes.py:170-223) and the window's
_preprocess_veh_state (apis/data_classes.py:34-39).  Returns index ranges, not window objects:
(k, x_start, x_end, t_start, t_end) per accepted vehicle, with the numpy slice semantics of
``data[x_start:x_end, t_start:t_end]`` left to the caller.  Pinned by tests/golden/select.npz.
"""
from __future__ import annotations

import numpy as np


def locate_windows(n_t_axis, t_axis, distances_along_fiber, x0, start_x_tracking, veh_states, t_axis_tracking,
                   dt, wlen_sw=8, length_sw=300, spatial_ratio=0.75, temporal_spacing=None):
    spacing = temporal_spacing if temporal_spacing else wlen_sw
    nsamp = int(wlen_sw / dt)
    half = nsamp // 2
    col = x0 - start_x_tracking
    n = len(veh_states)
    out = []
    for k in range(n):
        i0 = int(veh_states[k][col])
        if k < n - 1:  # a car close behind (the next pass arrives within the spacing)
            if t_axis_tracking[int(veh_states[k + 1][col])] - t_axis_tracking[i0] < spacing:
                continue
        if k > 0:  # a car close ahead (non-negative gap below the spacing)
            gap = t_axis_tracking[i0] - t_axis_tracking[int(veh_states[k - 1][col])]
            if 0 <= gap < spacing:
                continue
        t0 = t_axis_tracking[i0]
        best, c = None, 0
        for i in range(n_t_axis):  # argmin |t0 - t_axis|, first on ties
            d = abs(t0 - t_axis[i])
            if best is None or d < best:
                best, c = d, i
        if c < half or c + half > n_t_axis:
            continue
        sx_m = x0 - length_sw * spatial_ratio
        ex_m = sx_m + length_sw
        sx = int(np.abs(sx_m - distances_along_fiber).argmin())
        ex = int(np.abs(ex_m - distances_along_fiber).argmin())
        out.append((k, sx, ex, c - half, c - half + nsamp))
    return out


def veh_state_xt(veh_state, start_x_tracking, distance_along_fiber_tracking, t_axis_tracking):
    """apis/data_classes.py:34-39: tracked (distance, time) samples of one vehicle."""
    ok = [i for i in range(len(veh_state)) if not np.isnan(veh_state[i])]
    i0 = int(np.abs(start_x_tracking - distance_along_fiber_tracking).argmin())
    return (np.array([distance_along_fiber_tracking[i + i0] for i in ok]),
            np.array([t_axis_tracking[int(veh_state[i])] for i in ok]))
