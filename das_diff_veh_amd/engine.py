"""Batch engine behind the drop-in classes: windows -> device batches -> HIP kernels.

Windows are grouped by (window shape, gather rows, w, hop) so that each group is one launch of
each kernel; results come back in the caller's order.  Per group, the index tables are derived on
the device from the windows' trajectories (plan.DevicePlan / dvh_pass_geometry); the host computes
only what is per channel / time axis (the spatial searches and w, hop, nsamp from dt, with the
reference's errors).  Class stacks decide the windows' validity (data / ||data||_F,
apis/virtual_shot_gather.py:125) inside the stack launch (vsg_stack_validated) when norm or norm_amp
is on, and with a ||window||_F^2 launch otherwise.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
import sys
import threading

import numpy as np

from .device import default_device, to_device_f32, to_host_f64
from .plan import DevicePlan, VsgParams, pack_trajectories_checked, spatial_indices, window_lengths
from .vsg import StackSchedule, vsg_gathers, vsg_stack, vsg_stack_validated


@dataclasses.dataclass
class GatherAxes:
    """The axes of one pass's gather (post_processing_XCF, apis/virtual_shot_gather.py:130-132)."""
    gather_x_axis: np.ndarray
    gather_t_axis: np.ndarray


def _axes(win, prm: VsgParams):
    x = np.asarray(win.x_axis, dtype=np.float64)
    t = np.asarray(win.t_axis, dtype=np.float64)
    dt = t[1] - t[0]
    w, hop, _ = window_lengths(dt, prm)
    pv, st, en = spatial_indices(x, prm.pivot, prm.start_x, prm.end_x)
    if not (st <= pv < en):
        raise ValueError(f"unsupported gather geometry: start_idx={st}, pivot_idx={pv}, end_idx={en} "
                         f"(need start <= pivot < end)")
    return (en - st, w, hop), GatherAxes(x[st:en] - x[pv], (np.arange(w) - (w // 2)) * dt)


def _shared_or_stacked(arrays):
    """One 1-D axis when every window has the same one, else the [n, L] stack of them."""
    a0 = np.asarray(arrays[0], dtype=np.float64)
    if all(a is arrays[0] or np.array_equal(a0, a) for a in arrays[1:]):  # windows often share the axis object
        return a0
    return np.stack([np.asarray(a, dtype=np.float64) for a in arrays])


def _axes_all(windows, prm: VsgParams):
    """_axes of every window, evaluated once per distinct (channel axis, dt): notebook windows of one fiber
    section share their axes' values (the reference's per-window argmax searches give the same answer)."""
    memo, keys, axes = {}, [], []
    last = (None, None, None)  # (x_axis object, t_axis object, memo key): windows sharing the axis objects
    for w in windows:
        if w.x_axis is last[0] and w.t_axis is last[1] and last[2] is not None:
            mk = last[2]
        else:
            x = np.asarray(w.x_axis, dtype=np.float64)
            t = np.asarray(w.t_axis, dtype=np.float64)
            mk = (x.tobytes(), t[:2].tobytes()) if t.size >= 2 else None
            last = (w.x_axis, w.t_axis, mk)
        if mk is None or mk not in memo:
            r = _axes(w, prm)
            if mk is None:
                keys.append(r[0])
                axes.append(r[1])
                continue
            memo[mk] = r
        k, a = memo[mk]
        keys.append(k)
        axes.append(a)
    return keys, _OwnAxes(axes)


class _OwnAxes(list):
    """Every pass's GatherAxes; passes of one (channel axis, dt) share one memo entry, which an entry's first
    access replaces by the pass's own copy, so that every image still owns its axes (as the reference's
    per-window objects do) while the callers that read only a few entries (get_images reads the first) do not
    pay a copy per window."""

    def __init__(self, items):
        super().__init__(items)
        self._own = bytearray(len(self))

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        i = range(len(self))[i]
        a = super().__getitem__(i)
        if not self._own[i]:
            a = GatherAxes(a.gather_x_axis.copy(), a.gather_t_axis.copy())
            super().__setitem__(i, a)
            self._own[i] = 1
        return a

    def __setitem__(self, i, v):
        super().__setitem__(i, v)
        if isinstance(i, slice):
            for j in range(*i.indices(len(self))):
                self._own[j] = 1
        else:
            self._own[range(len(self))[i]] = 1

    def __iter__(self):
        return (self[i] for i in range(len(self)))


def _groups(windows, prm: VsgParams):
    """{(data shape, R, w, hop): window indices} and every pass's GatherAxes (host only)."""
    keys, axes = _axes_all(windows, prm) if windows else ((), ())
    groups = {}
    for i, (w, k) in enumerate(zip(windows, keys)):
        groups.setdefault((tuple(w.data.shape),) + k, []).append(i)
    return groups, axes


def _plan(windows, idx, key, prm: VsgParams, device):
    ws = [windows[i] for i in idx]
    trk, bad = pack_trajectories_checked([(w.veh_state_x, w.veh_state_t) for w in ws], device)
    plan = DevicePlan(_shared_or_stacked([w.x_axis for w in ws]), _shared_or_stacked([w.t_axis for w in ws]),
                      *trk, prm, key[0][0])
    return plan.check(bad)  # no device round trip (the H2D engine may be busy with the windows' staging)


def group_windows(windows, prm: VsgParams, device):
    """[(indices, DevicePlan)] per (data shape, R, w, hop) group, and every pass's GatherAxes."""
    groups, axes = _groups(windows, prm)
    return [(idx, _plan(windows, idx, key, prm, device)) for key, idx in groups.items()], axes


def _stage(windows, idx, device):
    """The group's windows to the device: host arrays through the pipelined staging on a background thread
    (their copies overlap the group's table work), device tensors stacked directly.  Returns a callable."""
    import torch

    from .device import stage_async
    arrs = [windows[i].data for i in idx]
    if not any(isinstance(a, torch.Tensor) for a in arrs):
        hosts = [np.asarray(a) for a in arrs]
        if all(h.dtype in (np.float32, np.float64) and h.ndim == 2 for h in hosts):
            return stage_async(hosts, device)
    return lambda: to_device_f32(arrs, device)


def _rows_of(batch_fn, idx, n, memo):
    """Callable giving rows idx of the staged batch batch_fn() (all n windows; evaluated once, kept in memo):
    the batch itself when idx is all of them in order."""
    def rows():
        import torch
        if "batch" not in memo:
            memo["batch"] = batch_fn()
        full = memo["batch"]
        if len(idx) == n and all(i == k for k, i in enumerate(idx)):
            return full
        return full[torch.as_tensor(np.asarray(idx, dtype=np.int64), device=full.device)]
    return rows


def gathers(windows, prm: VsgParams, device=None):
    """Per-pass gathers as float64 NumPy arrays, plus each pass's gather axes."""
    device = device or default_device()
    groups, axes = group_windows(windows, prm, device)
    res = [None] * len(windows)
    for idx, plan in groups:
        data = to_device_f32([windows[i].data for i in idx], device)
        g = to_host_f64(vsg_gathers(data, plan))
        for k, i in enumerate(idx):
            res[i] = g[k]
    return res, axes


# Opt-in (DVH_SWITCH_INTERVAL=<seconds>, default off): while any stacked() call is staging host windows, the
# interpreter's switch interval is lowered so that the staging thread's Python steps (chunk bookkeeping between its
# native copies) get the interpreter sooner while the calling thread groups and plans.  Process-wide state, so it is
# reference-counted under a lock: concurrent calls restore the caller's interval only when the last one ends.
_SWITCH = float(os.environ.get("DVH_SWITCH_INTERVAL", "0") or 0)
_SWITCH_LOCK = threading.Lock()
_SWITCH_STATE = {"depth": 0, "saved": None}


@contextlib.contextmanager
def _switch_interval():
    if _SWITCH <= 0:
        yield
        return
    with _SWITCH_LOCK:
        if _SWITCH_STATE["depth"] == 0:
            _SWITCH_STATE["saved"] = sys.getswitchinterval()
            sys.setswitchinterval(min(_SWITCH_STATE["saved"], _SWITCH))
        _SWITCH_STATE["depth"] += 1
    try:
        yield
    finally:
        with _SWITCH_LOCK:
            _SWITCH_STATE["depth"] -= 1
            if _SWITCH_STATE["depth"] == 0:
                sys.setswitchinterval(_SWITCH_STATE["saved"])


def stacked(windows, prm: VsgParams, slots=None, n_slot=1, device=None, chunk=8, counts=None):
    """Class-mean gathers [n_slot, R, w] (device tensor) over all windows, plus the gather axes.
    ``counts`` [n_slot]: the class sizes the means divide by (default: these windows' own; a rank of a
    sharded job passes the global ones, distributed.sharded_class_means)."""
    with _switch_interval():
        return _stacked(windows, prm, slots, n_slot, device, chunk, counts)


def _stacked(windows, prm, slots, n_slot, device, chunk, counts):
    device = device or default_device()
    slots = np.zeros(len(windows), dtype=np.int64) if slots is None else np.asarray(slots)
    counts = np.bincount(slots, minlength=n_slot) if counts is None else np.asarray(counts)
    # windows of one data shape (the notebooks' case) start their copies before anything else, in the caller's
    # order; a group takes its rows of the staged batch
    stagings = []  # every staging started here is waited for before an error leaves this call
    try:
        early = None
        if windows and len({np.shape(w.data) for w in windows}) == 1:
            early = _stage(windows, range(len(windows)), device)
            stagings.append(early)
        groups, axes = _groups(windows, prm)
        if len({key[1] for key in groups}) != 1:
            raise ValueError("operands could not be broadcast together: passes produce gathers of different shapes")
        # Windows whose time steps round to different w (499 / 500 on real axes) may share a class: sum(images)
        # keeps the first image's lag axis and adds the others' first min(w) lags (VirtualShotGather.__add__,
        # apis/virtual_shot_gather.py:195-199).  The stacks of the other lengths are formed apart and added so.
        w_of = {i: key[2] for key, idx in groups.items() for i in idx}
        first_w = {}
        for i, s in enumerate(slots):
            first_w.setdefault(int(s), w_of[i])
        if len(set(first_w.values())) > 1:
            raise ValueError("classes whose first passes have different lag lengths w: stack them in separate calls")
        w0 = next(iter(first_w.values()), None)
        if early is not None:
            memo = {}
            staged = [(idx, key, _rows_of(early, idx, len(windows), memo)) for key, idx in groups.items()]
        else:  # every group's window copies start first (background thread), the tables are formed meanwhile
            staged = []
            for key, idx in groups.items():
                staged.append((idx, key, _stage(windows, idx, device)))
                stagings.append(staged[-1][2])
        out = None
        for idx, key, data_fn in staged:
            plan = _plan(windows, idx, key, prm, device)
            data = data_fn()
            sched = StackSchedule(slots[idx], n_slot, chunk=chunk, counts=counts)
            fn = vsg_stack_validated if plan.flags & 6 else vsg_stack
            if key[2] == w0:
                out = fn(data, plan, sched, out=out, accumulate=out is not None)
            else:
                import torch
                part = fn(data, plan, sched)
                if out is None:
                    out = torch.zeros((n_slot, key[1], w0), dtype=torch.float32, device=part.device)
                m = min(w0, key[2])
                out[:, :, :m] += part[:, :, :m]
        return out, axes
    except BaseException:
        # a validation error after the copies started (geometry, shapes, trajectories): the background copies
        # finish before the error propagates, so none of them writes into memory released meanwhile and the
        # shared pinned buffers are free for the next staging
        for s in stagings:
            drain = getattr(s, "drain", None)
            if drain is not None:
                drain()
        raise


def stacked_sharded(windows, prm: VsgParams, slots=None, n_slot=1, group=None, device=None, chunk=8):
    """stacked() over the ranks of ``group``: every rank holds the same window list; each stacks its
    shard (distributed.shard_passes) with 1 / global class count weights and one all-reduce of the
    partial [n_slot, R, w] stacks gives every rank the class means.  Returns (stacks, axes of every
    window, this rank's pass indices)."""
    from .distributed import sharded_class_means
    import torch
    device = device or default_device()
    slots = np.zeros(len(windows), dtype=np.int64) if slots is None else np.asarray(slots, dtype=np.int64)
    keys, axes = zip(*[_axes(w, prm) for w in windows]) if windows else ((), ())
    if len({k[0] for k in keys}) != 1:
        raise ValueError("operands could not be broadcast together: passes produce gathers of different shapes")
    if len({k[1] for k in keys}) != 1:
        raise ValueError("the sharded class means need one lag length w (stacked() takes mixed ones)")
    # every pass is checked on every rank before sharding, so a bad pass raises the same error everywhere
    # instead of only on its owner (distributed.sharded_class_means also shares any error a rank hits)
    failed, _ = pass_failures(windows, prm)
    if failed:
        i = min(failed)
        raise ValueError(f"pass {i}: {failed[i]}")
    R, w = keys[0][:2]
    counts = np.bincount(slots, minlength=n_slot)

    def partial(mine, _weights):
        if mine.size == 0:
            return torch.zeros((n_slot, R, w), dtype=torch.float32, device=device)
        out, _ = stacked([windows[i] for i in mine], prm, slots[mine], n_slot, device, chunk, counts=counts)
        return out

    out, mine = sharded_class_means(partial, slots, n_slot, group)
    return out, list(axes), mine


def pass_failures(windows, prm: VsgParams):
    """Per-pass failure status of a batch, decided on the host before any launch (skip +
    count): {pass index: reason} for a gather geometry preprocessing_window cannot slice, the
    dt == 0.004 window-length mismatch, a trajectory interp1d (and dvh_pass_geometry) would reject
    (< 2 distinct finite tracked points), or a gather row count other than the batch's (that of its first
    good pass; another lag length w stacks as the reference's sum does).  Also returns every pass's GatherAxes
    (None for a failed one)."""
    failed, keys, axes = {}, {}, [None] * len(windows)
    for i, w in enumerate(windows):
        try:
            keys[i], axes[i] = _axes(w, prm)
        except ValueError as e:
            failed[i] = str(e)
            continue
        vx, vt = np.asarray(w.veh_state_x, dtype=np.float64), np.asarray(w.veh_state_t, dtype=np.float64)
        if vx.size < 2 or vx.size != vt.size or not np.all(np.isfinite(vx)) or np.unique(vx).size != vx.size:
            failed[i] = "trajectory needs >= 2 distinct finite tracked points (interp1d)"
    ok = [i for i in range(len(windows)) if i not in failed]
    if ok:  # gathers of another lag length w stack as sum(images) does; another row count cannot
        r0 = keys[ok[0]][0]
        for i in ok:
            if keys[i][0] != r0:
                failed[i] = f"gather rows R = {keys[i][0]} differ from the batch's {r0}"
    for i in failed:
        axes[i] = None
    return failed, axes


def stacked_checked(windows, prm: VsgParams, slots=None, n_slot=1, device=None, chunk=8):
    """stacked() with a failure status per pass instead of one per batch (skip + count).
    The reference raises on the first broken window and loses the whole class (a notebook cell dies);
    here the passes pass_failures() rejects are left out of their classes and reported, and the class
    means divide by the passes that were imaged.  Returns (stacks [n_slot, R, w] or None when no pass
    is left, axes per pass (None for a failed one), failed {pass index: reason})."""
    device = device or default_device()
    slots = np.zeros(len(windows), dtype=np.int64) if slots is None else np.asarray(slots, dtype=np.int64)
    failed, axes = pass_failures(windows, prm)
    ok = np.array([i for i in range(len(windows)) if i not in failed], dtype=np.int64)
    if ok.size == 0:
        return None, axes, failed
    counts = np.bincount(slots[ok], minlength=n_slot)
    out, _ = stacked([windows[i] for i in ok], prm, slots[ok], n_slot, device, chunk, counts=counts)
    return out, axes, failed
