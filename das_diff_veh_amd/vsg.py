"""Batched, device-resident virtual-shot-gather entry points (the hot path).

``windows`` is a CUDA (HIP) float32 tensor ``[n_pass, n_ch, n_t]`` (or any strided view whose time
axis is contiguous); tables come from :class:`das_diff_veh_amd.plan.VsgPlan`.  All calls are
stream-ordered on the current torch stream and never synchronise.

    scales = vsg_scales(windows, plan)                 # per-pass amplitude normalisation, [n, 2]
    g      = vsg_gathers(windows, plan, scales)        # per-pass gathers, [n, R, w]
    s      = vsg_stack(windows, plan, schedule)        # mean gather per class slot, [n_slot, R, w]
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .plan import VsgPlan

# Stack launches at w = 500 take a workspace for the per-pass table of pivot-slice spectra, so that the rows
# whose pivot slices it holds transform only their receivers (EngF500::spectra_tab); DVH_PIVOT_TABLE=0 runs
# them without it (every sub-window z = pivot + i receiver; A/B timing).
_TABLE = os.environ.get("DVH_PIVOT_TABLE", "1") != "0"


def spectra_workspace(plan: VsgPlan, device, cache: dict | None = None, table: bool | None = None):
    """The pivot-spectra workspace of a stack launch (None when the plan's w does not use one)."""
    if not (_TABLE if table is None else table):
        return None
    nbytes = int(_lib.load().dvh_vsg_stack_workspace(plan.n_pass, plan.w))
    if nbytes <= 0:
        return None
    if cache is not None:
        # one workspace per (device, stream): a launch on another stream must not overwrite the table a
        # launch still in flight on this one reads
        key = (str(device), torch.cuda.current_stream(device).cuda_stream)
        ws = cache.get(key)
        if ws is None or ws.numel() * 4 < nbytes:
            ws = cache[key] = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)
        return ws
    return torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)


def _check_windows(windows: torch.Tensor, plan: VsgPlan):
    if not windows.is_cuda:
        raise ValueError("windows must be a device tensor (the hot path has no CPU fallback)")
    if windows.dtype != torch.float32:
        raise TypeError("windows must be float32")
    if windows.dim() != 3 or windows.shape[0] != plan.n_pass:
        raise ValueError(f"windows must be [n_pass={plan.n_pass}, C, T], got {tuple(windows.shape)}")
    if windows.shape[1] < plan.n_ch or windows.shape[2] < plan.n_t or windows.stride(2) != 1:
        raise ValueError("windows smaller than the plan or time axis not contiguous")


def window_sumsq(windows: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """||window||_F^2 per pass (float64): the validity of the reference's data / ||data||_F
    (apis/virtual_shot_gather.py:125) -- NaN / inf anywhere or an all-zero window make the gather NaN."""
    if out is None:
        out = torch.empty(windows.shape[0], dtype=torch.float64, device=windows.device)
    _lib.call("dvh_window_sumsq", _lib.ptr(windows), windows.stride(0), windows.stride(1), windows.shape[0],
              windows.shape[1], windows.shape[2], _lib.ptr(out), _lib.stream_of(windows.device))
    return out


def vsg_scales(windows: torch.Tensor, plan: VsgPlan, out: torch.Tensor | None = None,
               win_sumsq: torch.Tensor | None = None, validity: bool = True) -> torch.Tensor:
    """Per-pass scales [n, 2].  ``win_sumsq`` (= window_sumsq(windows), a per-window property that
    callers imaging the same windows repeatedly compute once) also marks windows that are not
    finite or all zero, whose gathers are NaN in the reference (data / ||data||_F); it is computed
    here when not given, unless ``validity=False`` (the caller decides validity elsewhere, e.g.
    vsg_stack_validated) and norm or norm_amp is set (the raw mode's scale IS 1 / ||data||_F^2)."""
    _check_windows(windows, plan)
    pass_tab, seg_tab = plan.device_tables(windows.device)
    need = validity or not (plan.flags & 6)
    sumsq = window_sumsq(windows) if (win_sumsq is None and need) else win_sumsq
    if out is None:
        out = torch.empty((plan.n_pass, 2), dtype=torch.float32, device=windows.device)
    _lib.call("dvh_vsg_scales", _lib.ptr(windows), windows.stride(0), windows.stride(1), plan.n_pass,
              _lib.ptr(pass_tab), _lib.ptr(seg_tab), plan.R, plan.w, plan.hop, plan.flags, _lib.ptr(sumsq),
              _lib.ptr(out), _lib.stream_of(windows.device))
    return out


def vsg_gathers(windows: torch.Tensor, plan: VsgPlan, scales: torch.Tensor | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    _check_windows(windows, plan)
    if scales is None:
        scales = vsg_scales(windows, plan)
    pass_tab, seg_tab = plan.device_tables(windows.device)
    if out is None:
        out = torch.empty((plan.n_pass, plan.R, plan.w), dtype=torch.float32, device=windows.device)
    _lib.call("dvh_vsg_gathers", _lib.ptr(windows), windows.stride(0), windows.stride(1), plan.n_pass,
              _lib.ptr(pass_tab), _lib.ptr(seg_tab), plan.R, plan.w, plan.hop, plan.flags, _lib.ptr(scales),
              _lib.ptr(out), _lib.stream_of(windows.device))
    return out


class StackSchedule:
    """Passes sorted by class slot and cut into chunks that never straddle a slot.

    ``weights[p] = 1 / count[slot(p)]`` so the kernel's accumulation is directly the class mean
    (sum(images) / len(images)).  ``counts`` may be global counts (multi-GPU: each rank adds its
    share of the mean and an all-reduce sums them).
    """

    def __init__(self, slots, n_slot, chunk=8, counts=None, device=None):
        slots = np.asarray(slots, dtype=np.int64)
        if slots.size and (slots.min() < 0 or slots.max() >= n_slot):
            raise ValueError("slot id out of range")
        self.n_slot = n_slot
        order = np.argsort(slots, kind="stable")
        local = np.bincount(slots, minlength=n_slot)
        counts = local if counts is None else np.asarray(counts)
        with np.errstate(divide="ignore"):
            inv = np.where(counts > 0, 1.0 / np.maximum(counts, 1), 0.0)
        self.weights = inv[slots].astype(np.float32)
        chunks = []
        pos = 0
        for s in range(n_slot):
            n = int(local[s])
            for b in range(pos, pos + n, chunk):
                chunks.append((b, min(b + chunk, pos + n), s))
            pos += n
        self.order = order.astype(np.int32)
        self.chunk_tab = np.array(chunks, dtype=np.int32).reshape(-1, 3)
        self.counts = counts
        self._dev = {}

    def device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(device)
                                   for a in (self.order, self.chunk_tab, self.weights))
        return self._dev[key]


def vsg_stack(windows: torch.Tensor, plan: VsgPlan, schedule: StackSchedule, scales: torch.Tensor | None = None,
              out: torch.Tensor | None = None, accumulate: bool = False,
              win_sumsq: torch.Tensor | None = None, table: bool | None = None) -> torch.Tensor:
    """Class-mean gathers [n_slot, R, w]; with accumulate=True adds into ``out``.  ``scales`` come
    from vsg_scales (formed here with ``win_sumsq`` when not given).  ``table``: use the pivot-slice
    spectra table (default: on unless DVH_PIVOT_TABLE=0)."""
    _check_windows(windows, plan)
    pass_tab, seg_tab = plan.device_tables(windows.device)
    order, chunk_tab, weights = schedule.device_tables(windows.device)
    if out is None:
        out = torch.zeros((schedule.n_slot, plan.R, plan.w), dtype=torch.float32, device=windows.device)
    elif not accumulate:
        out.zero_()
    if scales is None:
        scales = vsg_scales(windows, plan, win_sumsq=win_sumsq)
    ws = spectra_workspace(plan, windows.device, getattr(plan, "_ws", None), table)
    _lib.call("dvh_vsg_stack", _lib.ptr(windows), windows.stride(0), windows.stride(1), plan.n_pass,
              _lib.ptr(pass_tab), _lib.ptr(seg_tab), plan.R, plan.w, plan.hop, plan.flags, _lib.ptr(scales),
              _lib.ptr(order), _lib.ptr(chunk_tab), int(chunk_tab.shape[0]), _lib.ptr(weights), _lib.ptr(out),
              _lib.ptr(ws), _lib.stream_of(windows.device))
    return out


def vsg_stack_validated(windows: torch.Tensor, plan: VsgPlan, schedule: StackSchedule, scales: torch.Tensor | None = None,
                        out: torch.Tensor | None = None, accumulate: bool = False,
                        work: torch.Tensor | None = None, scan: "UnitScan | None" = None) -> torch.Tensor:
    """vsg_stack plus the windows' validity in the same launch (dvh_vsg_stack_validated): every sample
    of every window [n_ch, n_t] is read once beside the correlations, and a class slot holding a
    pass whose window has a NaN / inf or is all zero becomes NaN -- the reference's data / ||data||_F
    (apis/virtual_shot_gather.py:125) -- without a separate ||window||_F pass.  Needs norm or norm_amp
    (the raw mode's scale is ||data||_F itself: use window_sumsq + vsg_stack).  ``work`` (optional):
    int32 device buffer of >= n_window + 2 elements, reused across calls.  ``scan``: the windows of a
    unit launch (UnitScan; default: one window per pass)."""
    _check_windows(windows, plan)
    if not (plan.flags & 6):
        raise ValueError("validated stacking needs norm or norm_amp; use window_sumsq + vsg_stack")
    if scan is None and windows.stride(0) == 0:
        raise ValueError("a unit launch (flat_units) validates its windows through a UnitScan")
    n_ch = windows.shape[1] if scan is None else scan.n_ch
    if n_ch < plan.R:
        raise ValueError("windows narrower than the gather")
    if scan is not None and scan.n_win and (scan.first_row.min() < 0 or scan.first_row.max() + scan.n_ch > windows.shape[1]):
        raise ValueError("scan windows reach outside the record rows")
    pass_tab, seg_tab = plan.device_tables(windows.device)
    order, chunk_tab, weights = schedule.device_tables(windows.device)
    if out is None:
        out = torch.zeros((schedule.n_slot, plan.R, plan.w), dtype=torch.float32, device=windows.device)
    elif not accumulate:
        out.zero_()
    if scales is None:
        scales = vsg_scales(windows, plan, validity=False)
    n_win = plan.n_pass if scan is None else scan.n_win
    if work is None or work.numel() < n_win + 2 or work.dtype != torch.int32:
        work = torch.empty(n_win + 2, dtype=torch.int32, device=windows.device)
    stab, uscan = (None, None) if scan is None else scan.device_tables(windows.device)
    ws = spectra_workspace(plan, windows.device, getattr(plan, "_ws", None))
    _lib.call("dvh_vsg_stack_validated", _lib.ptr(windows), windows.stride(0), windows.stride(1), plan.n_pass,
              n_ch, windows.shape[2], _lib.ptr(pass_tab), _lib.ptr(seg_tab), plan.R, plan.w, plan.hop,
              plan.flags, _lib.ptr(scales), _lib.ptr(order), _lib.ptr(chunk_tab), int(chunk_tab.shape[0]),
              schedule.n_slot, _lib.ptr(weights), _lib.ptr(out), _lib.ptr(stab), n_win, _lib.ptr(uscan),
              _lib.ptr(work), _lib.ptr(ws), _lib.stream_of(windows.device))
    return out


class UnitScan:
    """The windows a unit launch (plan.UnitPlan over flat_units) validates: window s = ``n_ch`` record
    rows from ``first_row[s]``; unit u takes the validity of window ``unit_window[u]``.  A pass imaged at
    several pivots is one window, read once per launch (the reference divides the pass's window by
    ||data||_F in every VirtualShotGather call, apis/virtual_shot_gather.py:125 -- the same value)."""

    def __init__(self, first_row, unit_window, n_ch):
        self.first_row = np.ascontiguousarray(first_row, dtype=np.int32)
        self.unit_window = np.ascontiguousarray(unit_window, dtype=np.int32)
        self.n_win, self.n_ch = int(self.first_row.size), int(n_ch)
        if self.unit_window.size and (self.unit_window.min() < 0 or self.unit_window.max() >= self.n_win):
            raise ValueError("unit window index out of range")
        self._dev = {}

    def device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = tuple(torch.from_numpy(a).to(device) for a in (self.first_row, self.unit_window))
        return self._dev[key]


def flat_units(windows: torch.Tensor, plan) -> torch.Tensor:
    """The launch view of a UnitPlan (plan.UnitPlan): windows [n, C, T] with contiguous (C, T) seen
    as n_unit copies of one flattened [n * C, T] record (pass stride 0); the plan's row0 / pivot
    already carry each unit's window offset q * C."""
    if not windows.is_cuda or windows.dtype != torch.float32 or windows.dim() != 3:
        raise ValueError("windows must be a float32 device tensor [n, C, T]")
    n, C, T = windows.shape
    if (n, C) != (plan.n_win, plan.win_ch) or T < plan.n_t:
        raise ValueError(f"windows {tuple(windows.shape)} do not match the plan ({plan.n_win}, {plan.win_ch}, {plan.n_t})")
    if windows.stride(2) != 1 or windows.stride(0) != C * windows.stride(1):
        raise ValueError("unit launches need windows contiguous in (channel, time)")
    return windows.as_strided((plan.n_pass, n * C, T), (0, windows.stride(1), 1))


def unit_sumsq(win_sumsq: torch.Tensor, plan) -> torch.Tensor:
    """Per-unit ||window||_F^2 from the per-window values (window_sumsq of the [n, C, T] windows)."""
    key = ("unit_window", str(win_sumsq.device))
    if key not in plan._dev:
        plan._dev[key] = torch.from_numpy(plan.unit_window).to(win_sumsq.device)
    return win_sumsq.index_select(0, plan._dev[key])
