"""Surface-wave window selection: one window per isolated pass.

SurfaceWaveSelector.locate_windows (apis/data_classes.py:170-223) splits into
  pass_table   the host index bookkeeping, O(n_passes): the crossing time of every tracked vehicle at
               column x0 - start_x_tracking, rejection of passes with a car behind (next crossing
               within temporal_spacing) or ahead (previous crossing 0 <= gap < temporal_spacing),
               the record sample nearest the crossing (argmin |t0 - t_axis|) and the boundary test,
               and the channel range nearest x0 - length_sw * spatial_ratio .. + length_sw; the
               reference's float64 expressions, its int() truncation and its error on an untracked
               crossing (``int(nan)`` raises ValueError) are kept;
  cut_windows  the copies themselves: every accepted pass's [channels, samples] block of the record
               cut into one contiguous device batch by dvh_cut_windows, ready for the imaging kernels.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .device import default_device
from .plan import py_slice


def pass_table(t_axis, distances_along_fiber, x0, start_x_tracking, veh_states, t_axis_tracking, dt, wlen_sw=8,
               length_sw=300, spatial_ratio=0.75, temporal_spacing=None):
    """-> (ks, (x_start, x_end), t_starts, t_ends): accepted vehicle indices and their slice bounds."""
    spacing = temporal_spacing if temporal_spacing else wlen_sw
    nsamp = int(wlen_sw / dt)
    half = nsamp // 2
    vs = np.asarray(veh_states)
    n = len(vs)
    if n == 0:
        return np.zeros(0, np.int64), (0, 0), np.zeros(0, np.int64), np.zeros(0, np.int64)
    col = vs[:, x0 - start_x_tracking]  # the reference's column index (an int, as numpy demands)
    if not np.all(np.isfinite(col)):
        raise ValueError("cannot convert float NaN to integer")
    idx = np.trunc(col).astype(np.int64)  # int(v[x0_idx])
    tt = np.asarray(t_axis_tracking)
    tc = tt[idx]
    behind = np.zeros(n, bool)
    behind[:-1] = tc[1:] - tc[:-1] < spacing
    gap = np.full(n, -1.0)
    gap[1:] = tc[1:] - tc[:-1]
    ahead = (spacing > gap) & (gap >= 0)
    ahead[0] = False
    ks, t0s = [], []
    t_axis = np.asarray(t_axis)
    for k in np.flatnonzero(~behind & ~ahead):
        c = int(np.abs(tc[k] - t_axis).argmin())
        if c < half or c + half > t_axis.size:
            continue
        ks.append(int(k))
        t0s.append(c - half)
    sx_m = x0 - length_sw * spatial_ratio
    ex_m = sx_m + length_sw
    dist = np.asarray(distances_along_fiber)
    xr = (int(np.abs(sx_m - dist).argmin()), int(np.abs(ex_m - dist).argmin()))
    t0s = np.asarray(t0s, dtype=np.int64)
    return np.asarray(ks, dtype=np.int64), xr, t0s, t0s + nsamp


def _dtype_code(t):
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.float64:
        return 1
    raise TypeError("the record must be float32 or float64")


def cut_windows(record, x_range, t_starts, t_ends, out_dtype=None):
    """Device batches of data[x_start:x_end, t_start:t_end] (numpy slice semantics) for every pass.

    ``record`` is a 2-D device tensor.  Returns (batches, where): {length: contiguous batch} (all but a
    pass clipped at the record's end share one length) and, per pass, its (length, row) in them."""
    if not (isinstance(record, torch.Tensor) and record.is_cuda and record.dim() == 2):
        raise ValueError("record must be a 2-D device tensor (no CPU fallback)")
    if record.stride(1) != 1:
        record = record.contiguous()
    n_rows, n_t = record.shape
    out_dtype = out_dtype or record.dtype
    xs, xl = (int(v) for v in py_slice(x_range[0], x_range[1], n_rows))
    ts, tl = py_slice(np.asarray(t_starts, np.int64), np.asarray(t_ends, np.int64), n_t)
    dev = record.device
    where = [None] * len(ts)
    batches = {}
    for length in sorted(set(int(v) for v in tl)):
        members = np.flatnonzero(tl == length)
        batch = batches[length] = torch.empty((members.size, xl, length), dtype=out_dtype, device=dev)
        if batch.numel():
            starts = torch.as_tensor(ts[members], dtype=torch.int64, device=dev)
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            _lib.call("dvh_cut_windows", _lib.ptr(record), _dtype_code(record), n_rows, record.stride(0), n_t,
                      _lib.ptr(starts), members.size, xs, xl, length, _lib.ptr(batch), _dtype_code(batch),
                      _lib.ptr(status), _lib.stream_of(dev))
            if int(status.item()) != 0:
                raise IndexError("a window lies outside the record")
        for j, m in enumerate(members):
            where[m] = (length, j)
    return batches, where


def record_on_device(data, device=None):
    """The record as a device tensor (host float arrays are uploaded once, dtype kept)."""
    if isinstance(data, torch.Tensor) and data.is_cuda:
        return data
    host = np.asarray(data.detach().cpu() if isinstance(data, torch.Tensor) else data)
    if host.dtype not in (np.float32, np.float64):
        host = host.astype(np.float64)
    return torch.from_numpy(np.ascontiguousarray(host)).to(device or default_device())
