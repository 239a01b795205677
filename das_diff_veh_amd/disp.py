"""Batched dispersion (f-v) transform on device: host tables + the three dvh_disp_* kernels.

Host side does only integer/float64 bookkeeping with the reference's own expressions:
  nf = 2 ** (1 + ceil(log(nt, 2))), nk = 2 ** (1 + ceil(log(nch, 2)))      modules/utils.py:239-240
  fft_f = arange(-nf/2, nf/2) / nf / dt, fft_k = arange(-nk/2, nk/2) / nk / dx  :242-243
  queries (k = f / v, f) sorted ascending per frequency (interp2d.__call__), clamped to the grid
  FITPACK degree-1 basis h = (t_hi - q, q - t_lo) / (t_hi - t_lo)
  savgol_filter(25, 4, mode='interp') as a linear operator: interior taps (savgol_coeffs) and the
  two edge polynomial-fit matrices (_fit_edge)
Every FLOP on the data runs in the kernels (das_diff_veh_amd/csrc/dvh_disp.hip).
"""
from __future__ import annotations

import math
import os

import numpy as np
import scipy.signal
import torch

from . import _lib


def fk_sizes(nch, nt):
    nf = 2 ** (1 + math.ceil(math.log(nt, 2)))
    nk = 2 ** (1 + math.ceil(math.log(nch, 2)))
    return nf, nk


def fk_axes(nch, nt, dx, dt):
    nf, nk = fk_sizes(nch, nt)
    return np.arange(-nf / 2, nf / 2) / nf / dt, np.arange(-nk / 2, nk / 2) / nk / dx


def _intervals(grid, q):
    """fpbisp: clamp to [grid[0], grid[-1]] and pick l with grid[l] <= q < grid[l+1], l <= n - 2."""
    q = np.clip(q, grid[0], grid[-1])
    l = np.clip(np.searchsorted(grid, q, side="right") - 1, 0, grid.size - 2)
    return q, l


def savgol_operator(window_length=25, polyorder=4):
    """(h, E_left, E_right) of scipy.signal.savgol_filter(..., mode='interp') as linear maps."""
    h = scipy.signal.savgol_coeffs(window_length, polyorder)
    half = window_length // 2
    vfit = np.vander(np.arange(window_length, dtype=np.float64), polyorder + 1)
    pinv = np.linalg.pinv(vfit)
    el = np.vander(np.arange(0, half, dtype=np.float64), polyorder + 1) @ pinv
    er = np.vander(np.arange(window_length - half, window_length, dtype=np.float64), polyorder + 1) @ pinv
    return h[::-1].copy(), el, er


class DispPlan:
    """Everything the kernels need for one (nch, nt, dx, dt, freqs, vels) geometry."""

    def __init__(self, nch, nt, dx, dt, freqs, vels, sg_window=25, sg_order=4, full_grid=False):
        self.nch, self.nt, self.dx, self.dt = int(nch), int(nt), float(dx), float(dt)
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.vels = np.asarray(vels, dtype=np.float64)
        self.nF, self.nV = self.freqs.size, self.vels.size
        if self.nF < sg_window:
            raise ValueError("If mode is 'interp', window_length must be less than or equal to the size of x.")
        nf, nk = fk_sizes(nch, nt)
        self.nf, self.nk = nf, nk
        fft_f, fft_k = fk_axes(nch, nt, dx, dt)
        self.fft_f, self.fft_k = fft_f, fft_k

        # frequency direction: one scalar query per output column
        fq, j0 = _intervals(fft_f, self.freqs)
        ones = np.ones(self.nV)
        kq = np.stack([np.sort(np.divide(ones * fr, self.vels), kind="mergesort") for fr in self.freqs])
        kqc, m0 = _intervals(fft_k, kq)
        self._m0 = m0
        if full_grid:
            j_lo, j_hi, m_lo, m_hi = 0, nf - 1, 0, nk - 1
        else:
            j_lo, j_hi = int(j0.min()), int(j0.max()) + 1
            m_lo, m_hi = int(m0.min()), int(m0.max()) + 1
        self.j_lo, self.m_lo = j_lo, m_lo
        self.n_fb = j_hi - j_lo + 1
        self.n_kb = m_hi - m_lo + 1
        flo, fhi = fft_f[j0], fft_f[j0 + 1]
        fy = 1.0 / (fhi - flo)
        self.fj = (j0 - j_lo).astype(np.int32)
        self.fw = np.stack([fy * (fhi - fq), fy * (fq - flo)], axis=1)
        self.kq = np.ascontiguousarray(kq)
        self.kgrid = np.ascontiguousarray(fft_k[m_lo:m_hi + 1])
        self.kmin, self.kmax = float(fft_k[0]), float(fft_k[-1])

        # time-DFT twiddles for the needed bins nu = (j - nf/2) mod nf
        nu = (np.arange(j_lo, j_hi + 1) - nf // 2) % nf
        t = np.arange(nt)
        ang = 2.0 * np.pi * ((np.outer(t, nu) % nf) / nf)
        wt = np.empty((nt, 2 * self.n_fb))
        wt[:, 0::2] = np.cos(ang)
        wt[:, 1::2] = -np.sin(ang)
        self.wt = wt

        # channel-contraction block matrix [[Er, -Ei], [Ei, Er]] for kappa = (m - nk/2) mod nk
        self.MT = 16 * ((self.n_kb + 15) // 16)
        self.K2 = 4 * ((2 * self.nch + 3) // 4)
        kappa = (np.arange(m_lo, m_hi + 1) - nk // 2) % nk
        th = 2.0 * np.pi * ((np.outer(kappa, np.arange(nch)) % nk) / nk)
        er, ei = np.cos(th), -np.sin(th)
        a = np.zeros((2 * self.MT, self.K2))
        a[:self.n_kb, :nch] = er
        a[:self.n_kb, nch:2 * nch] = -ei
        a[self.MT:self.MT + self.n_kb, :nch] = ei
        a[self.MT:self.MT + self.n_kb, nch:2 * nch] = er
        self.atab = a

        h, el, er_ = savgol_operator(sg_window, sg_order)
        self.sgl = sg_window
        self.sg = np.concatenate([h, el.ravel(), er_.ravel()])
        self.mk = (m0 - m_lo).astype(np.int32)  # FITPACK interval of every (f, v) query, compact-grid rows
        self._cells = None
        self._dev = {}

    # f-v blocks of the frequency-tiled kernel: 256 threads, 4 velocities, tiles of <= 200 outputs with a
    # 12-sample halo (one tile when the whole axis fits the block)
    TILE_THREADS, TILE_VT, TILE_PAD = 256, 4, 12

    def cell_tables(self):
        """Per (velocity chunk, frequency tile) block of dvh_disp_fv_cells: the FK cells its bilinear stencils
        read -- rows m, m + 1 of columns j, j + 1 for every (f, v) it samples -- column-major (each column's
        rows lo..hi contiguous), and per (f, v) the compact indices of (m, j) and (m, j + 1) with m.
        Returns a dict of numpy tables (cached), or None when a block would not fit."""
        if self._cells is not None:
            return self._cells or None
        T, VT, pad = self.TILE_THREADS, self.TILE_VT, self.TILE_PAD
        nF, nV = self.nF, self.nV
        nt = 1 if nF <= T else -(-nF // 200)
        TO = (-(-nF // nt) + 3) & ~3
        ok = nF >= self.sgl
        nvc = -(-nV // VT)
        n_ct = nvc * nt
        qidx = np.zeros((n_ct, T, VT, 4), dtype=np.int32)
        offs, ncell = [], np.zeros(n_ct, dtype=np.int32)
        for t in range(nt):
            f_lo, f_hi = t * TO, min(nF, t * TO + TO)
            s0, s1 = max(0, f_lo - pad), min(nF, max(f_hi + pad, self.sgl))
            ok &= (s1 - s0 <= T) and (nt == 1 or f_hi - f_lo >= pad + 1)
            fs = np.arange(s0, s1)
            for c in range(nvc):
                vs = np.arange(c * VT, min(nV, c * VT + VT))
                M = self.mk[np.ix_(fs, vs)].astype(np.int64)
                J = np.broadcast_to(self.fj[fs].astype(np.int64)[:, None], M.shape)
                cols = np.concatenate([J.ravel(), J.ravel() + 1])
                rows = np.concatenate([M.ravel(), M.ravel()])
                ucol, inv = np.unique(cols, return_inverse=True)
                lo = np.full(ucol.size, np.iinfo(np.int64).max)
                hi = np.full(ucol.size, -1)
                np.minimum.at(lo, inv, rows)
                np.maximum.at(hi, inv, rows + 1)
                cnt = hi - lo + 1
                start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
                col_of = np.repeat(ucol, cnt)
                row_of = np.arange(cnt.sum()) - np.repeat(start, cnt) + np.repeat(lo, cnt)
                ct = c * nt + t
                offs.append((row_of * self.n_fb + col_of).astype(np.int32))
                ncell[ct] = offs[-1].size
                c0, c1 = np.searchsorted(ucol, J), np.searchsorted(ucol, J + 1)
                qidx[ct, :fs.size, :vs.size, 0] = start[c0] + M - lo[c0]
                qidx[ct, :fs.size, :vs.size, 1] = start[c1] + M - lo[c1]
                qidx[ct, :fs.size, :vs.size, 2] = M
        # offs was filled tile-major: reorder to ct = c * nt + t
        order = [c * nt + t for t in range(nt) for c in range(nvc)]
        by_ct = [None] * n_ct
        for k, ct in enumerate(order):
            by_ct[ct] = offs[k]
        max_cell = int(ncell.max())
        ok &= max_cell <= 8192
        if not ok:
            self._cells = {}
            return None
        cell_off = np.zeros((n_ct, max_cell), dtype=np.int32)
        for ct, o in enumerate(by_ct):
            cell_off[ct, :o.size] = o
        self._cells = dict(TO=TO, n_tile=nt, max_cell=max_cell, cell_off=cell_off, n_cell=ncell, qidx=qidx)
        return self._cells

    def mfma_tables(self):
        """dvh_disp_fv_mfma's per-(f, v) tables (cached): the FITPACK degree-1 weights of every clamped query
        on its interval m, hx[f][v] = (fx * (khi - q), fx * (q - klo)) with fx = 1 / (khi - klo) -- the
        expressions the sampling kernels evaluate, so the values are bit-identical -- and the compact cell
        offset cb[f][v] = m * n_fb + fj[f]."""
        if getattr(self, "_mfma", None) is None:
            q = np.clip(self.kq, self.kmin, self.kmax)
            m = self.mk.astype(np.int64)
            klo, khi = self.kgrid[m], self.kgrid[m + 1]
            fx = 1.0 / (khi - klo)
            hx = np.stack([fx * (khi - q), fx * (q - klo)], axis=-1)
            cb = (m * self.n_fb + self.fj.astype(np.int64)[:, None]).astype(np.int32)
            self._mfma = dict(hx=np.ascontiguousarray(hx), cb=np.ascontiguousarray(cb))
        return self._mfma

    def tables(self, device):
        key = str(device)
        if key not in self._dev:
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            self._dev[key] = dict(wt=t(self.wt), atab=t(self.atab), kgrid=t(self.kgrid), kq=t(self.kq),
                                  fj=t(self.fj), fw=t(self.fw), sg=t(self.sg))
        return self._dev[key]


def _check(data, plan):
    if not data.is_cuda or data.dtype != torch.float32:
        raise ValueError("data must be a float32 device tensor (no CPU fallback)")
    if data.dim() != 3 or data.shape[1] != plan.nch or data.shape[2] != plan.nt or data.stride(2) != 1:
        raise ValueError(f"data must be [B, {plan.nch}, {plan.nt}] with a contiguous time axis")


def fk_grid(data, plan: DispPlan, norm=False, slots=None, weights=None, n_slot=None):
    """|FK| on the plan's compact grid: [B, n_kb, n_fb], or per-slot weighted sums [n_slot, ...]."""
    _check(data, plan)
    dev = data.device
    tb = plan.tables(dev)
    B = data.shape[0]
    st = _lib.stream_of(dev)
    scale = None
    if norm:
        scale = torch.empty(B * plan.nch, dtype=torch.float32, device=dev)
        _lib.call("dvh_disp_row_l1", _lib.ptr(data), data.stride(0), data.stride(1), B, plan.nch, plan.nt,
                  _lib.ptr(scale), st)
    D = torch.empty((B * plan.nch, 2 * plan.n_fb), dtype=torch.float64, device=dev)
    _lib.call("dvh_disp_tdft", _lib.ptr(data), data.stride(0), data.stride(1), B, plan.nch, plan.nt,
              _lib.ptr(tb["wt"]), plan.n_fb, _lib.ptr(scale), _lib.ptr(D), st)
    if slots is None:
        FK = torch.empty((B, plan.n_kb, plan.n_fb), dtype=torch.float64, device=dev)
        sl = wt = None
    else:
        slots = np.asarray(slots, dtype=np.int64)
        if n_slot is None or slots.shape != (B,) or (B and (slots.min() < 0 or slots.max() >= n_slot)):
            raise ValueError("fk_grid: one class slot in [0, n_slot) per gather")
        FK = torch.zeros((n_slot, plan.n_kb, plan.n_fb), dtype=torch.float64, device=dev)
        sl = torch.as_tensor(slots.astype(np.int32), device=dev)
        wt = torch.as_tensor(np.asarray(weights, dtype=np.float32), device=dev)
    _lib.call("dvh_disp_fk", _lib.ptr(D), B, plan.nch, plan.n_fb, _lib.ptr(tb["atab"]), plan.MT, plan.K2,
              plan.n_kb, _lib.ptr(FK), _lib.ptr(sl), _lib.ptr(wt), 0 if n_slot is None else int(n_slot), st)
    return FK


def _use_cells(plan: DispPlan, B: int) -> bool:
    """The cell-staged tiled kernel for batches that fill the chip (>= 4 096 blocks); few images (the
    bench's class stacks) keep the per-image kernel.  DVH_FV_CELLS=0 / 1 forces it off / on (A/B)."""
    env = os.environ.get("DVH_FV_CELLS")
    if env is not None:
        return env != "0" and plan.cell_tables() is not None
    if "DVH_FV_TILE" in os.environ or "DVH_FV_G" in os.environ:  # A/B of the dvh_disp_fv kernels
        return False
    nt = 1 if plan.nF <= DispPlan.TILE_THREADS else -(-plan.nF // 200)
    if B * nt * -(-plan.nV // DispPlan.TILE_VT) < 4096:
        return False
    return plan.cell_tables() is not None


def _use_mfma(plan: DispPlan, B: int) -> bool:
    """The MFMA-filter kernel (dvh_disp_fv_mfma) where it applies: savgol window 25, nF >= 32, a compact FK
    grid of at most 8 192 bins.  DVH_FV_MFMA=0 / 1 forces it off / on (A/B)."""
    ok = plan.sgl == 25 and plan.nF >= 32 and plan.n_kb * plan.n_fb <= 8192
    env = os.environ.get("DVH_FV_MFMA")
    if env is not None:
        return env != "0" and ok
    if any(k in os.environ for k in ("DVH_FV_TILE", "DVH_FV_G", "DVH_FV_CELLS")):  # A/B of the other kernels
        return False
    return ok and B * -(-plan.nV // 64) >= MFMA_MIN_BLOCKS


MFMA_MIN_BLOCKS = 512  # (64-velocity block, image) pairs: two blocks per CU


def fv_from_fk(FK, plan: DispPlan, out=None):
    dev = FK.device
    tb = plan.tables(dev)
    B = FK.shape[0]
    if out is None:
        out = torch.empty((B, plan.nV, plan.nF), dtype=torch.float32, device=dev)
    if _use_mfma(plan, B):
        key = ("mfma", str(dev))
        if key not in plan._dev:
            mt = plan.mfma_tables()
            plan._dev[key] = {k: torch.from_numpy(v).to(dev) for k, v in mt.items()}
        mt = plan._dev[key]
        G = int(os.environ.get("DVH_FV_MG", "0"))
        _lib.call("dvh_disp_fv_mfma", _lib.ptr(FK), B, plan.n_kb, plan.n_fb, _lib.ptr(mt["hx"]), _lib.ptr(mt["cb"]),
                  plan.nF, plan.nV, _lib.ptr(tb["fw"]), _lib.ptr(tb["sg"]), plan.sgl, G, _lib.ptr(out),
                  _lib.stream_of(dev))
        return out
    if _use_cells(plan, B):
        key = ("cells", str(dev))
        if key not in plan._dev:
            ct = plan.cell_tables()
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
            plan._dev[key] = dict(ct, cell_off=t(ct["cell_off"]), n_cell=t(ct["n_cell"]), qidx=t(ct["qidx"]))
        c = plan._dev[key]
        _lib.call("dvh_disp_fv_cells", _lib.ptr(FK), B, plan.n_kb, plan.n_fb, _lib.ptr(tb["kgrid"]), plan.kmin,
                  plan.kmax, _lib.ptr(tb["kq"]), plan.nF, plan.nV, _lib.ptr(tb["fw"]), _lib.ptr(tb["sg"]), plan.sgl,
                  c["TO"], c["n_tile"], DispPlan.TILE_VT, c["max_cell"], _lib.ptr(c["cell_off"]), _lib.ptr(c["n_cell"]),
                  _lib.ptr(c["qidx"]), _lib.ptr(out), _lib.stream_of(dev))
        return out
    _lib.call("dvh_disp_fv", _lib.ptr(FK), B, plan.n_kb, plan.n_fb, _lib.ptr(tb["kgrid"]), plan.kmin, plan.kmax,
              _lib.ptr(tb["kq"]), plan.nF, plan.nV, _lib.ptr(tb["fj"]), _lib.ptr(tb["fw"]), _lib.ptr(tb["sg"]),
              plan.sgl, _lib.ptr(out), _lib.stream_of(dev))
    return out


def fv_maps(data, plan: DispPlan, norm=False):
    """map_fv for every gather of the batch: [B, Nvel, Nfreq] float32 (rows = sorted-query order)."""
    return fv_from_fk(fk_grid(data, plan, norm=norm), plan)


def fv_class_means(data, plan: DispPlan, slots, n_slot, norm=False, counts=None):
    """Mean f-v image per class slot (sum(disps) / len): the transform after |FK| is linear, so the
    per-pass |FK| grids are averaged on device and sampled once per slot."""
    slots = np.asarray(slots, dtype=np.int64)
    counts = np.bincount(slots, minlength=n_slot) if counts is None else np.asarray(counts)
    w = np.where(counts[slots] > 0, 1.0 / np.maximum(counts[slots], 1), 0.0)
    return fv_from_fk(fk_grid(data, plan, norm=norm, slots=slots, weights=w, n_slot=n_slot), plan)
