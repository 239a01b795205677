"""Batch engine behind the drop-in classes: windows -> device batches -> HIP kernels.

Windows are grouped by (window shape, gather rows, w, hop) so that each group is one launch of
each kernel; results come back in the caller's order.
"""
from __future__ import annotations

import numpy as np
import torch

from .device import default_device, to_device_f32, to_host_f64
from .plan import VsgParams, VsgPlan, pass_geometry
from .vsg import StackSchedule, vsg_gathers, vsg_scales, vsg_stack


def _data_shape(win):
    d = win.data
    return tuple(d.shape)


def group_windows(windows, prm: VsgParams):
    geoms = [pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, prm) for w in windows]
    groups = {}
    for i, (w, g) in enumerate(zip(windows, geoms)):
        key = (_data_shape(w), g.end_idx - g.start_idx, g.w, g.hop)
        groups.setdefault(key, []).append(i)
    out = []
    for key, idx in groups.items():
        shape = key[0]
        out.append((idx, VsgPlan([geoms[i] for i in idx], prm, shape[0], shape[1])))
    return out, geoms


def gathers(windows, prm: VsgParams, device=None):
    """Per-pass gathers as float64 NumPy arrays, plus each pass's (x_axis, t_axis)."""
    device = device or default_device()
    groups, geoms = group_windows(windows, prm)
    res = [None] * len(windows)
    for idx, plan in groups:
        data = to_device_f32([windows[i].data for i in idx], device)
        g = to_host_f64(vsg_gathers(data, plan))
        for k, i in enumerate(idx):
            res[i] = g[k]
    return res, geoms


def stacked(windows, prm: VsgParams, slots=None, n_slot=1, device=None, chunk=8):
    """Class-mean gathers [n_slot, R, w] (device tensor) over all windows."""
    device = device or default_device()
    slots = np.zeros(len(windows), dtype=np.int64) if slots is None else np.asarray(slots)
    counts = np.bincount(slots, minlength=n_slot)
    groups, geoms = group_windows(windows, prm)
    keys = {(plan.R, plan.w) for _, plan in groups}
    if len(keys) != 1:
        raise ValueError("operands could not be broadcast together: passes produce gathers of different shapes")
    out = None
    for idx, plan in groups:
        data = to_device_f32([windows[i].data for i in idx], device)
        sched = StackSchedule(slots[idx], n_slot, chunk=chunk, counts=counts)
        out = vsg_stack(data, plan, sched, out=out, accumulate=out is not None)
    return out, geoms
