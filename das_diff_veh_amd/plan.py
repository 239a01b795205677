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


# ------------------------------------------------------------------------------------------------
# Sliding pivots: one pass window imaged at many pivots along the fiber.
#
# The reference images a window at one pivot per VirtualShotGather call
# (apis/virtual_shot_gather.py:183-192); sliding the pivot along the fiber is the caller looping
# over pivots with start_x = pivot - a, end_x = pivot + a.  Here every (pass, pivot) pair is one
# "unit" of a single launch.  The kernels address channel ch of unit u's window as
# win + ch * ch_stride: with the windows [n, C, T] contiguous in (C, T), window q's channel c is
# channel q * C + c of one flattened [n * C, T] record, so a unit carries row0 / pivot offset by
# q * C and the launch sees pass_stride = 0 (das_diff_veh_amd.vsg.flat_units).  No ABI change.

def sliding_pivots(x_axis, pivot_ch, half_aperture):
    """Spatial indices of gathers centred on channels pivot_ch with start_x / end_x = pivot -/+ a:
    (pivot_idx, start_idx, end_idx) arrays with the reference's expressions
    (argmax(x >= pivot), argmax(x >= start_x), argmin|x - end_x|; preprocessing_window :111-126)."""
    x_axis = np.asarray(x_axis, dtype=np.float64)
    piv = x_axis[np.asarray(pivot_ch, dtype=np.int64)]
    ge = lambda v: np.argmax(x_axis[None, :] >= v[:, None], axis=1)  # noqa: E731
    return (ge(piv), ge(piv - half_aperture), np.abs(x_axis[None, :] - (piv + half_aperture)[:, None]).argmin(axis=1),
            piv)


def sliding_geometry(x_axis, t_axis, veh_state_x, veh_state_t, spatial, prm: VsgParams):
    """seg tables of one pass at every pivot of ``spatial`` (from sliding_pivots), vectorised over
    pivots and rows with pass_geometry's expressions (bit-identical tables: tests/test_host.py).

    Returns (seg [J, R, 2, 2] int64, full [J] bool): ``full`` marks the pivots whose every row has
    full-length time slices on both sides (the vehicle crosses the aperture inside the window)."""
    x_axis = np.asarray(x_axis, dtype=np.float64)
    t_axis = np.asarray(t_axis, dtype=np.float64)
    pivot_idx, start_idx, end_idx, piv = spatial
    R = int(end_idx[0] - start_idx[0])
    if np.any(end_idx - start_idx != R):
        raise ValueError("sliding pivots must share the gather row count")
    f = interp1d_extrap(veh_state_x, veh_state_t)
    dt = t_axis[1] - t_axis[0]
    w = int(prm.wlen / dt)
    nsamp = int(prm.time_window_to_xcorr // dt)
    T = t_axis.size
    rows = start_idx[:, None] + np.arange(R)[None, :]                  # [J, R]
    # every expression is elementwise, so it is evaluated once per channel and gathered per
    # (pivot, row): f(x[rows]) == f(x)[rows], f(pivot) == f(x)[pivot channel] (pivots sit on channels)
    fx = f(x_axis)
    fp = f(piv)
    seg = np.zeros((len(piv), R, 2, 2), dtype=np.int64)
    pt = first_true_ge(t_axis, fp + prm.delta_t)[:, None]
    ti = first_true_ge(t_axis, fx + prm.delta_t)[rows]
    shared = rows <= pivot_idx[:, None]
    a = np.where(shared, pt, ti)
    seg[:, :, 0, 0], seg[:, :, 0, 1] = py_slice(a, a + nsamp, T)
    if prm.include_other_side:
        pt = first_true_ge(t_axis, fp + (-prm.delta_t))[:, None]
        ti = first_true_ge(t_axis, fx - prm.delta_t)[rows]
        shared = rows >= pivot_idx[:, None]
        b = np.where(shared, pt, ti)
        seg[:, :, 1, 0], seg[:, :, 1, 1] = py_slice(b - nsamp, b, T)
        full = np.all(seg[:, :, :, 1] == nsamp, axis=(1, 2))
    else:
        full = np.all(seg[:, :, 0, 1] == nsamp, axis=1)
    if w < 2:
        raise ValueError(f"correlation window too short: w={w}")
    return seg, full


def sliding_full(x_axis, t_axis, veh_state_x, veh_state_t, spatial, prm: VsgParams):
    """sliding_geometry's ``full`` mask in O(C + J): per-channel slice lengths and prefix counts of
    short slices, so that only the pivots a pass crosses get [R, 2, 2] tables."""
    x_axis = np.asarray(x_axis, dtype=np.float64)
    t_axis = np.asarray(t_axis, dtype=np.float64)
    pivot_idx, start_idx, end_idx, piv = spatial
    f = interp1d_extrap(veh_state_x, veh_state_t)
    dt = t_axis[1] - t_axis[0]
    nsamp = int(prm.time_window_to_xcorr // dt)
    T = t_axis.size
    fx, fp = f(x_axis), f(piv)

    def short_prefix(ti, sgn):
        a = ti if sgn > 0 else ti - nsamp
        bad = (py_slice(a, a + nsamp, T)[1] != nsamp).astype(np.int64)
        return np.concatenate([[0], np.cumsum(bad)])

    def shared_ok(sgn):
        pt = first_true_ge(t_axis, fp + sgn * prm.delta_t)
        a = pt if sgn > 0 else pt - nsamp
        return py_slice(a, a + nsamp, T)[1] == nsamp

    cf = short_prefix(first_true_ge(t_axis, fx + prm.delta_t), 1)
    full = shared_ok(1) & (cf[end_idx] - cf[pivot_idx + 1] == 0)          # forward rows pivot+1..end-1
    if prm.include_other_side:
        co = short_prefix(first_true_ge(t_axis, fx - prm.delta_t), -1)
        full &= shared_ok(-1) & (co[pivot_idx] - co[start_idx] == 0)       # other-side rows start..pivot-1
    return full


class UnitPlan(VsgPlan):
    """A launch over (window, pivot) units: VsgPlan tables with row0 / pivot offset by window * C.

    ``unit_window[u]`` / ``unit_pivot[u]`` name each unit's window and pivot (index into the
    spatial tables); ``n_ch`` of the plan is the flattened record's n * C channels."""

    def __init__(self, seg_tab, unit_window, unit_pivot, spatial, prm: VsgParams, n_win, n_ch, n_t, dt, piv_ch=None):
        pivot_idx, start_idx, end_idx, piv = spatial
        self.R = int(end_idx[0] - start_idx[0])
        self.w = int(prm.wlen / dt)
        self.hop = int(self.w * (1 - 0.5))
        self.nsamp = int(prm.time_window_to_xcorr // dt)
        self.prm = prm
        self.flags = prm.flags
        self.unit_window = np.asarray(unit_window, dtype=np.int64)
        self.unit_pivot = np.asarray(unit_pivot, dtype=np.int64)
        self.n_pass = self.unit_window.size
        if self.n_pass == 0:
            raise ValueError("empty batch")
        self.n_win, self.win_ch = int(n_win), int(n_ch)
        self.pivots = np.asarray(piv_ch) if piv_ch is not None else None
        self.n_ch, self.n_t = int(n_win) * int(n_ch), int(n_t)
        off = self.unit_window * n_ch
        self.pass_tab = np.stack([start_idx[self.unit_pivot] + off, pivot_idx[self.unit_pivot] + off],
                                 axis=1).astype(np.int32)
        self.seg_tab = np.ascontiguousarray(seg_tab, dtype=np.int32)
        if self.n_ch >= 2 ** 31:
            raise ValueError("flattened record exceeds int32 channel indices")
        assert self.seg_tab.shape == (self.n_pass, self.R, 2, 2)
        assert self.seg_tab.min() >= 0 and (self.seg_tab[..., 0] + self.seg_tab[..., 1]).max() <= n_t
        self.geoms = None
        self._dev = {}

    @classmethod
    def sliding(cls, x_axis, t_axis, trajectories, pivot_ch, half_aperture, prm: VsgParams, full_only=True):
        """Units (q, j) for every window q (trajectories[q] = (veh_state_x, veh_state_t)) and pivot
        channel pivot_ch[j]; with full_only only the pivots the vehicle crosses inside the window."""
        spatial = sliding_pivots(x_axis, pivot_ch, half_aperture)
        segs, uw, up = [], [], []
        for q, (vx, vt) in enumerate(trajectories):
            if full_only:
                j = np.nonzero(sliding_full(x_axis, t_axis, vx, vt, spatial, prm))[0]
                if j.size == 0:
                    segs.append(np.zeros((0, int(spatial[2][0] - spatial[1][0]), 2, 2), dtype=np.int64))
                    continue
                seg = sliding_geometry(x_axis, t_axis, vx, vt, tuple(a[j] for a in spatial), prm)[0]
            else:
                j = np.arange(spatial[0].size)
                seg = sliding_geometry(x_axis, t_axis, vx, vt, spatial, prm)[0]
            segs.append(seg)
            uw.append(np.full(j.size, q))
            up.append(j)
        if not uw:
            raise ValueError("empty batch: no pass crosses a pivot inside its window")
        t_axis = np.asarray(t_axis, dtype=np.float64)
        return cls(np.concatenate(segs), np.concatenate(uw), np.concatenate(up), spatial, prm, len(trajectories),
                   len(x_axis), t_axis.size, t_axis[1] - t_axis[0], piv_ch=pivot_ch)
