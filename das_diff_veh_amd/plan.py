"""Host-side index tables for the batched VSG kernels (float64, bit-exact with the reference).

An off-by-one here is not a rounding error but a different gather, so every index is derived with
the reference's own float64 expressions:

  preprocessing_window            apis/virtual_shot_gather.py:111-126
      f = interp1d(veh_state_x, veh_state_t, fill_value='extrapolate')
      pivot_idx = argmax(x >= pivot); start_idx = argmax(x >= start_x); end_idx = argmin|x - end_x|
      pt = argmax(t >= f(pivot) + delta_t);  nsamp = int(time_window_to_xcorr // dt)
  XCORR_* window bookkeeping       modules/utils.py:255-257, 292-295
      w = int(wlen / dt); hop = int(w * 0.5); nwin = (nt - w) // hop + 1
  xcorr_two_traces_based_on_traj   apis/virtual_shot_gather.py:24-35
      t_idx = argmax(t >= f(x_row) +- delta_t); slices [t_idx, t_idx + nsamp) / [t_idx - nsamp, t_idx)
Python slice semantics (negative starts wrap, ends clamp) are reproduced exactly; the kernels only
ever see (start, length) pairs inside [0, T].
"""
from __future__ import annotations

import dataclasses

import numpy as np


def interp1d_extrap(xp, yp):
    """Linear interpolation with linear extrapolation, with the arithmetic of
    scipy.interpolate.interp1d(kind='linear', fill_value='extrapolate') (SciPy 1.15 ``_call_linear``)."""
    order = np.argsort(xp, kind="mergesort")
    x = np.asarray(xp, dtype=np.float64)[order]
    y = np.asarray(yp, dtype=np.float64)[order]
    if x.size < 2:
        raise ValueError("trajectory needs at least two tracked points")

    def f(xq):
        xq = np.asarray(xq, dtype=np.float64)
        i = np.clip(np.searchsorted(x, xq), 1, x.size - 1)
        lo = i - 1
        slope = (y[i] - y[lo]) / (x[i] - x[lo])
        return slope * (xq - x[lo]) + y[lo]

    return f


def first_true_ge(t_axis, t):
    """np.argmax(t_axis >= t) for every t (0 when no sample qualifies, NaN included)."""
    t = np.asarray(t, dtype=np.float64)
    if t_axis.size > 1 and np.all(np.diff(t_axis) > 0):
        i = np.searchsorted(t_axis, t, side="left")
        return np.where(i >= t_axis.size, 0, i)
    return np.argmax(t_axis[None, :] >= np.atleast_1d(t)[:, None], axis=1).reshape(t.shape)


def py_slice(a, b, n):
    """(start, length) of x[a:b] for len(x) == n, Python semantics, step 1."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    a = np.where(a < 0, np.maximum(a + n, 0), np.minimum(a, n))
    b = np.where(b < 0, np.maximum(b + n, 0), np.minimum(b, n))
    return a, np.maximum(b - a, 0)


@dataclasses.dataclass(frozen=True)
class VsgParams:
    """Keyword surface of construct_shot_gather (apis/virtual_shot_gather.py:165-166) + VirtualShotGather."""
    pivot: float = 635
    start_x: float = 530
    end_x: float = 680
    wlen: float = 2
    norm: bool = True
    norm_amp: bool = True
    time_window_to_xcorr: float = 4
    delta_t: float = 1
    include_other_side: bool = False

    @property
    def flags(self):
        return (1 if self.include_other_side else 0) | (2 if self.norm else 0) | (4 if self.norm_amp else 0)


@dataclasses.dataclass
class PassGeometry:
    w: int
    hop: int
    nsamp: int
    dt: float
    start_idx: int
    pivot_idx: int
    end_idx: int
    seg: np.ndarray          # [R, 2 sides, 2] (start, length)
    gather_x_axis: np.ndarray
    gather_t_axis: np.ndarray


def pass_geometry(x_axis, t_axis, veh_state_x, veh_state_t, prm: VsgParams) -> PassGeometry:
    x_axis = np.asarray(x_axis, dtype=np.float64)
    t_axis = np.asarray(t_axis, dtype=np.float64)
    f = interp1d_extrap(veh_state_x, veh_state_t)
    dt = t_axis[1] - t_axis[0]
    w = int(prm.wlen / dt)
    w_alloc = int(prm.wlen // dt)
    if w != w_alloc:
        # xcorr_two_traces_based_on_traj allocates int(wlen // dt) columns for rows of int(wlen / dt)
        # samples; the reference raises on the assignment / concatenate (dt == 0.004).
        raise ValueError(f"could not broadcast input array from shape (1,{w}) into shape ({w_alloc},): "
                         f"int(wlen // dt) != int(wlen / dt) for dt = {dt!r}")
    hop = int(w * (1 - 0.5))
    nsamp = int(prm.time_window_to_xcorr // dt)
    T = t_axis.size
    pivot_idx = int(np.argmax(x_axis >= prm.pivot))
    start_idx = int(np.argmax(x_axis >= prm.start_x))
    end_idx = int(np.abs(x_axis - prm.end_x).argmin())
    if not (start_idx <= pivot_idx < end_idx):
        raise ValueError(f"unsupported gather geometry: start_idx={start_idx}, pivot_idx={pivot_idx}, "
                         f"end_idx={end_idx} (need start <= pivot < end)")
    if w < 2 or hop < 1:
        raise ValueError(f"correlation window too short: w={w}")
    rows = np.arange(start_idx, end_idx)
    R = rows.size
    seg = np.zeros((R, 2, 2), dtype=np.int64)
    fp = f(prm.pivot)

    # forward side (construct_shot_gather)
    pt = int(first_true_ge(t_axis, fp + prm.delta_t))
    shared = rows <= pivot_idx
    a, L = py_slice(pt, pt + nsamp, T)
    seg[shared, 0, 0], seg[shared, 0, 1] = a, L
    traj = ~shared
    if traj.any():
        ti = first_true_ge(t_axis, f(x_axis[rows[traj]]) + prm.delta_t)
        a, L = py_slice(ti, ti + nsamp, T)
        seg[traj, 0, 0], seg[traj, 0, 1] = a, L

    # other side (construct_shot_gather_other_side: delta_t -> -delta_t, windows end at the index)
    if prm.include_other_side:
        pt = int(first_true_ge(t_axis, fp + (-prm.delta_t)))
        shared = rows >= pivot_idx
        a, L = py_slice(pt - nsamp, pt, T)
        seg[shared, 1, 0], seg[shared, 1, 1] = a, L
        traj = ~shared
        if traj.any():
            t = f(x_axis[rows[traj]])
            ti = first_true_ge(t_axis, t - prm.delta_t)
            a, L = py_slice(ti - nsamp, ti, T)
            seg[traj, 1, 0], seg[traj, 1, 1] = a, L

    gx = x_axis[start_idx:end_idx] - x_axis[pivot_idx]
    gt = (np.arange(w) - (w // 2)) * dt
    return PassGeometry(w, hop, nsamp, dt, start_idx, pivot_idx, end_idx, seg, gx, gt)


class VsgPlan:
    """Index tables of one kernel launch: uniform (R, w, hop) over all passes."""

    def __init__(self, geoms, prm: VsgParams, n_ch: int, n_t: int):
        if not geoms:
            raise ValueError("empty batch")
        g0 = geoms[0]
        self.R = g0.end_idx - g0.start_idx
        self.w, self.hop, self.nsamp = g0.w, g0.hop, g0.nsamp
        for g in geoms:
            if (g.end_idx - g.start_idx, g.w, g.hop) != (self.R, self.w, self.hop):
                raise ValueError("passes of one batch must share (rows, w, hop); group them first")
            if g.end_idx > n_ch:
                raise ValueError("gather rows beyond the window")
        self.prm = prm
        self.flags = prm.flags
        self.n_pass = len(geoms)
        self.n_ch, self.n_t = n_ch, n_t
        self.geoms = geoms
        self.pass_tab = np.array([[g.start_idx, g.pivot_idx] for g in geoms], dtype=np.int32)
        self.seg_tab = np.stack([g.seg for g in geoms]).astype(np.int32)  # [n, R, 2, 2]
        assert self.seg_tab.min() >= 0 and (self.seg_tab[..., 0] + self.seg_tab[..., 1]).max() <= n_t
        self._dev = {}

    @classmethod
    def from_trajectories(cls, x_axes, t_axes, veh_xs, veh_ts, prm: VsgParams, n_ch: int, n_t: int):
        geoms = [pass_geometry(x, t, vx, vt, prm) for x, t, vx, vt in zip(x_axes, t_axes, veh_xs, veh_ts)]
        return cls(geoms, prm, n_ch, n_t)

    def nwin(self):
        L = self.seg_tab[..., 1].astype(np.int64)
        return np.where(L >= self.w, (L - self.w) // self.hop + 1, 0)

    def algorithmic_bytes(self, out_rows=0):
        """Bytes a launch must move: every receiver sample under a sub-window, each distinct pivot
        sample of a pass once, and out_rows gather rows of w fp32 written."""
        nw = self.nwin()
        sides = 2 if self.prm.include_other_side else 1
        cov = np.where(nw > 0, (nw - 1) * self.hop + self.w, 0)[:, :, :sides]
        rcv = 4 * int(cov.sum())
        piv = 0
        for p in range(self.n_pass):
            a = self.seg_tab[p, :, :sides, 0].ravel()
            c = cov[p].ravel()
            iv = sorted((int(x), int(x + y)) for x, y in zip(a, c) if y > 0)
            tot, cur_s, cur_e = 0, None, None
            for s, e in iv:
                if cur_e is None or s > cur_e:
                    if cur_e is not None:
                        tot += cur_e - cur_s
                    cur_s, cur_e = s, e
                else:
                    cur_e = max(cur_e, e)
            if cur_e is not None:
                tot += cur_e - cur_s
            piv += 4 * tot
        return rcv + piv + 4 * out_rows * self.w

    def device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            import torch
            self._dev[key] = (torch.from_numpy(np.ascontiguousarray(self.pass_tab)).to(device),
                              torch.from_numpy(np.ascontiguousarray(self.seg_tab)).to(device))
        return self._dev[key]
