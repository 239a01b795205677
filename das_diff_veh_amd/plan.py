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


def seg_nwin(seg_tab, w, hop):
    """Sub-windows per (pass, row, side): (L - w) // hop + 1, or 0 when the slice is shorter than w."""
    L = np.asarray(seg_tab)[..., 1].astype(np.int64)
    return np.where(L >= w, (L - w) // hop + 1, 0)


def seg_algorithmic_bytes(seg_tab, w, hop, sides, out_rows=0):
    """Bytes a launch must move for the tables seg_tab [n, R, 2, 2]: 4 B x every receiver sample under
    a sub-window, 4 B x each distinct pivot sample of a pass (the union of its rows' slices), and
    out_rows gather rows of w fp32 written."""
    seg = np.asarray(seg_tab)
    n = seg.shape[0]
    nw = seg_nwin(seg, w, hop)[:, :, :sides]
    cov = np.where(nw > 0, (nw - 1) * hop + w, 0).astype(np.int64)
    rcv = 4 * int(cov.sum())
    # union of the pivot-channel intervals [a, a + cov) per pass: sort by start, running max of ends
    a = seg[:, :, :sides, 0].reshape(n, -1).astype(np.int64)
    e = a + cov.reshape(n, -1)
    o = np.argsort(a, axis=1, kind="stable")
    a, e = np.take_along_axis(a, o, 1), np.take_along_axis(e, o, 1)
    prev = np.concatenate([np.full((n, 1), np.iinfo(np.int64).min), np.maximum.accumulate(e, axis=1)[:, :-1]], 1)
    piv = 4 * int(np.maximum(e - np.maximum(a, prev), 0).sum())
    return rcv + piv + 4 * out_rows * w


def spatial_indices(x_axis, pivot, start_x, end_x):
    """(pivot_idx, start_idx, end_idx) of preprocessing_window (apis/virtual_shot_gather.py:111-126):
    argmax(x >= pivot), argmax(x >= start_x), argmin |x - end_x|; x_axis [C] with scalars, or [n, C]
    with scalars or per-pass [n] values."""
    x = np.asarray(x_axis, dtype=np.float64)
    if x.ndim == 1:
        return (int(np.argmax(x >= pivot)), int(np.argmax(x >= start_x)), int(np.abs(x - end_x).argmin()))
    col = lambda v: np.asarray(v, dtype=np.float64).reshape(-1, 1)  # noqa: E731
    return (np.argmax(x >= col(pivot), axis=1), np.argmax(x >= col(start_x), axis=1),
            np.abs(x - col(end_x)).argmin(axis=1))


def window_lengths(dt, prm):
    """(w, hop, nsamp) for a sample interval dt (XCORR_* bookkeeping, modules/utils.py:255-257), with the
    reference's ValueError when int(wlen // dt) != int(wlen / dt) (dt == 0.004)."""
    w = int(prm.wlen / dt)
    w_alloc = int(prm.wlen // dt)
    if w != w_alloc:
        raise ValueError(f"could not broadcast input array from shape (1,{w}) into shape ({w_alloc},): "
                         f"int(wlen // dt) != int(wlen / dt) for dt = {dt!r}")
    if w < 2:
        raise ValueError(f"correlation window too short: w={w}")
    return w, int(w * (1 - 0.5)), int(prm.time_window_to_xcorr // dt)


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
        if self.seg_tab.min() < 0 or (self.seg_tab[..., 0] + self.seg_tab[..., 1]).max() > n_t:
            raise ValueError("time slices outside the window: the passes' t_axis does not match the window's "
                             f"{n_t} samples")
        self._dev = {}
        self._ws = {}  # (device, stream) -> stack-launch workspace (vsg.spectra_workspace)

    @classmethod
    def from_trajectories(cls, x_axes, t_axes, veh_xs, veh_ts, prm: VsgParams, n_ch: int, n_t: int):
        geoms = [pass_geometry(x, t, vx, vt, prm) for x, t, vx, vt in zip(x_axes, t_axes, veh_xs, veh_ts)]
        return cls(geoms, prm, n_ch, n_t)

    def nwin(self):
        return seg_nwin(self.seg_tab, self.w, self.hop)

    def algorithmic_bytes(self, out_rows=0):
        """Bytes a launch must move: every receiver sample under a sub-window, each distinct pivot
        sample of a pass once, and out_rows gather rows of w fp32 written."""
        return seg_algorithmic_bytes(self.seg_tab, self.w, self.hop, 2 if self.prm.include_other_side else 1,
                                     out_rows)

    def device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            import torch
            self._dev[key] = (torch.from_numpy(np.ascontiguousarray(self.pass_tab)).to(device),
                              torch.from_numpy(np.ascontiguousarray(self.seg_tab)).to(device))
        return self._dev[key]


class DevicePlan:
    """The index tables of one launch derived ON THE DEVICE from the passes' trajectories
    (dvh_pass_geometry, bit-identical to pass_geometry): the per-pass, per-row float64 work of
    preprocessing_window / xcorr_two_traces_based_on_traj (apis/virtual_shot_gather.py:111-126, 24-35)
    runs as a kernel on the launch's stream, so a pipeline forms each batch's tables where it images it.

    The host keeps only what is per channel axis, not per pass: the spatial searches (pivot / start /
    end index) and (w, hop, nsamp) from dt, with the reference's errors.  Trajectories are device
    float64 tensors [n, L] (padded; ``trk_len`` [n] int32 valid points, strictly ascending x).
    ``x_axis`` / ``t_axis`` are shared 1-D arrays or per-pass [n, C] / [n, T] arrays.  Same interface
    as VsgPlan for the vsg_* entry points (``device_tables``); ``derive()`` (re)launches the kernel,
    e.g. after the trajectory tensors were refilled for a new batch."""

    def __init__(self, x_axis, t_axis, trk_x, trk_t, trk_len, prm: VsgParams, n_ch: int, pivot_x=None,
                 start_x=None, end_x=None, derive=True, seg_out=None):
        import torch
        self.prm, self.flags = prm, prm.flags
        x = np.asarray(x_axis, dtype=np.float64)
        t = np.asarray(t_axis, dtype=np.float64)
        n = int(trk_x.shape[0])
        if n == 0:
            raise ValueError("empty batch")
        if trk_x.dtype != torch.float64 or trk_t.dtype != torch.float64 or not trk_x.is_cuda:
            raise ValueError("trajectories must be float64 device tensors [n, L]")
        if trk_t.shape != trk_x.shape or trk_x.stride(1) != 1 or trk_t.stride() != trk_x.stride():
            raise ValueError("trk_x / trk_t must share a row-contiguous [n, L] layout")
        dts = t[..., 1] - t[..., 0]
        lens = {window_lengths(float(d), prm) for d in np.atleast_1d(dts)}
        if len(lens) != 1:
            raise ValueError("passes of one batch must share (w, hop, nsamp); group them first")
        self.w, self.hop, self.nsamp = lens.pop()
        piv = np.full(n, float(prm.pivot)) if pivot_x is None else np.asarray(pivot_x, dtype=np.float64)
        if x.shape[-1] != n_ch or (x.ndim == 2 and x.shape[0] != n) or (t.ndim == 2 and t.shape[0] != n):
            raise ValueError("x_axis / t_axis must be shared 1-D axes or one row per pass")
        sx = prm.start_x if start_x is None else np.asarray(start_x, dtype=np.float64)
        ex = prm.end_x if end_x is None else np.asarray(end_x, dtype=np.float64)
        if x.ndim == 1 and pivot_x is None and start_x is None and end_x is None:
            pv, st, en = spatial_indices(x, prm.pivot, sx, ex)
        else:
            pv, st, en = spatial_indices(np.broadcast_to(x, (n, x.shape[-1])), piv, sx, ex)
        pv, st, en = (np.broadcast_to(np.asarray(v), (n,)) for v in (pv, st, en))
        if not np.all((st <= pv) & (pv < en)):
            raise ValueError("unsupported gather geometry (need start <= pivot < end)")
        R = en - st
        if np.any(R != R[0]):
            raise ValueError("passes of one batch must share (rows, w, hop); group them first")
        self.R = int(R[0])
        self.n_pass, self.n_ch, self.n_t = n, int(n_ch), int(t.shape[-1])
        if int(en.max()) > self.n_ch:
            raise ValueError("gather rows beyond the window")
        dev = trk_x.device
        from .device import upload
        self.pass_tab, self.pivot_x, self._x, self._t = upload(
            [np.stack([st, pv], 1).astype(np.int32), piv, x, t], dev)
        self.trk_x, self.trk_t = trk_x, trk_t
        self.trk_len = trk_len.to(device=dev, dtype=torch.int32)
        if seg_out is not None:  # caller-owned table buffer (e.g. shared by a pipeline's batches)
            if seg_out.dtype != torch.int32 or seg_out.numel() < n * self.R * 4 or not seg_out.is_contiguous():
                raise ValueError("seg_out must be a contiguous int32 buffer of >= n * R * 4 elements")
            self.seg_tab = seg_out.view(-1)[:n * self.R * 4].view(n, self.R, 2, 2)
        else:
            self.seg_tab = torch.empty((n, self.R, 2, 2), dtype=torch.int32, device=dev)
        self.status = torch.empty(n, dtype=torch.int32, device=dev)
        self.geoms = None
        self._ws = {}  # (device, stream) -> stack-launch workspace, shared by the slices (same-stream launches are ordered)
        if derive:
            self.derive()

    def derive(self):
        """Launch dvh_pass_geometry on the current stream (asynchronous)."""
        from . import _lib
        x_stride = self.n_ch if self._x.dim() == 2 else 0
        t_stride = self.n_t if self._t.dim() == 2 else 0
        _lib.call("dvh_pass_geometry", _lib.ptr(self._x), x_stride, _lib.ptr(self._t), t_stride, self.n_t,
                  _lib.ptr(self.trk_x), _lib.ptr(self.trk_t), self.trk_x.stride(0), _lib.ptr(self.trk_len),
                  _lib.ptr(self.pivot_x), _lib.ptr(self.pass_tab), self.n_pass, self.R, float(self.prm.delta_t),
                  self.nsamp, 1 if self.prm.include_other_side else 0, _lib.ptr(self.seg_tab), _lib.ptr(self.status),
                  _lib.stream_of(self.trk_x.device))
        return self

    def device_tables(self, device=None):
        return self.pass_tab, self.seg_tab

    def slice(self, a, b):
        """Passes [a, b) as a plan of their own whose tables are views of this plan's: one derive()
        of the whole plan forms every slice's tables in a single launch (a pipeline's batches), and a
        slice's derive() re-forms only its passes."""
        import copy
        if not 0 <= a < b <= self.n_pass:
            raise ValueError(f"slice [{a}, {b}) outside the plan's {self.n_pass} passes")
        sub = copy.copy(self)
        sub.n_pass = b - a
        for name in ("pass_tab", "pivot_x", "trk_x", "trk_t", "trk_len", "seg_tab", "status"):
            setattr(sub, name, getattr(self, name)[a:b])
        if self._x.dim() == 2:
            sub._x = self._x[a:b]
        if self._t.dim() == 2:
            sub._t = self._t[a:b]
        sub.geoms = None
        return sub

    def check(self, host_status=None):
        """Raise like interp1d would for passes whose trajectory could not be evaluated: from host_status
        (pack_trajectories_checked's, the same rule) when given, else from the kernel's (synchronises)."""
        st = self.status.cpu().numpy() if host_status is None else np.asarray(host_status)
        bad = np.nonzero(st)[0]
        if bad.size:
            raise ValueError(f"passes {bad.tolist()[:8]}: trajectory needs >= 2 strictly ascending tracked points")
        return self

    def host_seg_tab(self):
        return self.seg_tab.cpu().numpy()

    def nwin(self):
        return seg_nwin(self.host_seg_tab(), self.w, self.hop)

    def algorithmic_bytes(self, out_rows=0):
        return seg_algorithmic_bytes(self.host_seg_tab(), self.w, self.hop,
                                     2 if self.prm.include_other_side else 1, out_rows)


def pack_trajectories(trajectories, device):
    """[(veh_state_x, veh_state_t), ...] -> padded float64 device tensors (trk_x, trk_t [n, L]) and
    trk_len [n] int32, the layout dvh_pass_geometry reads.  Each trajectory is ordered by x with a
    stable sort first, as interp1d does (its mergesort of the abscissae)."""
    return pack_trajectories_checked(trajectories, device)[0]


def pack_trajectories_checked(trajectories, device):
    """pack_trajectories, plus each pass's status as dvh_pass_geometry forms it (1: fewer than 2 points or not
    strictly ascending once sorted, NaN included), computed here from the same sorted rows so that
    DevicePlan.check() needs no device round trip."""
    n = len(trajectories)
    lens = np.array([len(vx) for vx, _ in trajectories], dtype=np.int64)
    L = max(1, int(lens.max()) if n else 1)
    one = n > 0 and int(lens.min()) == L  # every pass the same length: the block is the padded layout itself
    tx = None if one else np.zeros((n, L))
    tt = None if one else np.zeros((n, L))
    ln = lens.astype(np.int32)
    bad = (lens < 2).astype(np.int32)
    # trajectories of one length are ordered together (one [m, k] block per length: the tracker's passes share
    # a handful of lengths): a row-wise stable argsort equals each row's mergesort, and rows already ascending
    # (the tracker's output) are copied as they are
    for k in np.unique(lens):
        idx = np.flatnonzero(lens == k)
        vx = np.array([np.asarray(trajectories[i][0], dtype=np.float64) for i in idx]).reshape(idx.size, k)
        vt = np.array([np.asarray(trajectories[i][1], dtype=np.float64) for i in idx]).reshape(idx.size, k)
        asc = vx[:, 1:] > vx[:, :-1]
        if k > 1 and not np.all(asc):
            o = np.argsort(vx, axis=1, kind="stable")
            vx, vt = np.take_along_axis(vx, o, 1), np.take_along_axis(vt, o, 1)
            asc = vx[:, 1:] > vx[:, :-1]
        if k > 1:
            bad[idx] |= ~np.all(asc, axis=1)  # a pair not strictly ascending (NaN included)
        if one:
            tx, tt = vx, vt
        else:
            tx[idx, :k], tt[idx, :k] = vx, vt
    from .device import upload
    return tuple(upload([tx, tt, ln], device)), bad


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
        self.spatial, self.dt = spatial, dt
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
        if self.seg_tab.min() < 0 or (self.seg_tab[..., 0] + self.seg_tab[..., 1]).max() > n_t:
            raise ValueError("time slices outside the window: the passes' t_axis does not match the window's "
                             f"{n_t} samples")
        self.geoms = None
        self._dev = {}
        self._ws = {}  # (device, stream) -> stack-launch workspace (vsg.spectra_workspace)

    @classmethod
    def concat(cls, plans):
        """One launch over the units of several plans on the SAME windows and pivots (e.g. batches of new
        trajectories over one resident pool): their tables concatenated.  More units per launch means
        more passes per (class, pivot) slot chunk, i.e. fewer inverse transforms and stack atomics."""
        p0 = plans[0]
        for p in plans[1:]:
            if (p.n_win, p.win_ch, p.n_t, p.R, p.w, p.hop, p.flags) != (p0.n_win, p0.win_ch, p0.n_t, p0.R, p0.w, p0.hop,
                                                                         p0.flags):
                raise ValueError("plans of one launch must share windows, gather shape and flags")
            if not all(np.array_equal(a, b) for a, b in zip(p.spatial, p0.spatial)):
                raise ValueError("plans of one launch must share their pivots")
        return cls(np.concatenate([p.seg_tab for p in plans]), np.concatenate([p.unit_window for p in plans]),
                   np.concatenate([p.unit_pivot for p in plans]), p0.spatial, p0.prm, p0.n_win, p0.win_ch, p0.n_t,
                   p0.dt, p0.pivots)

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
