"""Bootstrap / convergence resampling on the device.

The reference recomputes every virtual shot gather of every resample from scratch
(``bootstrap_disp``, apis/imaging_classes.py:8-48, called 30 x 60 times per class by the notebooks'
``convergence_test``, imaging_diff_speed.ipynb#cell30).  Here:

  1. the per-pass gathers of all windows are computed once (``dvh_vsg_gathers``) and kept in HBM
     (``GatherCache``; 96 KB per pass for the notebook geometry);
  2. a resample's stack -- ``sum(images) / len(images)`` of its ``random.sample`` draw -- is a gather-
     mean over the cached rows the dispersion image reads (``dvh_select_mean``, summed in draw order);
  3. the f-v images of all resamples go through the batched dispersion kernels in one launch each;
  4. every (resample, mode) ridge is walked by one wave (``dvh_ridge``): extract_ridge_ref_idx,
     modules/utils.py:621-678, with its strict velocity window, first-index argmax and savgol(25, 2).

Random draws use Python's ``random`` exactly as the reference does (``random.sample(range(1, n), k)``,
index 0 never drawn), so seeding ``random`` reproduces the reference's resamples.
"""
from __future__ import annotations

import random
import time

import numpy as np
import torch

from . import _lib
from .device import default_device, to_device_f32
from .disp import DispPlan, fk_grid, fv_from_fk, savgol_operator
from .plan import VsgParams, VsgPlan, pass_geometry
from .vsg import vsg_gathers

FREQS = np.arange(0.8, 25, 0.1)   # Dispersion defaults of compute_disp_image (apis/virtual_shot_gather.py:247)
VELS = np.arange(200, 1200)
_SG_RIDGE = None


def _sg_ridge():
    global _SG_RIDGE
    if _SG_RIDGE is None:
        h, el, er = savgol_operator(25, 2)
        _SG_RIDGE = np.concatenate([h, el.ravel(), er.ravel()])
    return _SG_RIDGE


def ridges(fv, freqs, vels, freq_lb, freq_ub, ref_freq_idx=None, sigma=25, vel_max=400, ref_vel=None,
           return_picks=False):
    """extract_ridge_ref_idx (modules/utils.py:621-678) for every image of ``fv`` [B, Nvel, Nfreq]
    (device float32, rows in the map's order = ``vels`` reversed) on the band lb <= f < ub.
    ``ref_freq_idx`` indexes the band; ``ref_vel`` is a callable of frequency (or an array over
    the band).  Returns float64 [B, n_band] on the host (and the raw picks before the smoothing
    with return_picks=True)."""
    return ridges_finish(ridges_launch(fv, freqs, vels, freq_lb, freq_ub, ref_freq_idx, sigma, vel_max, ref_vel,
                                       return_picks))


def ridges_finish(pending):
    """Host results of a ridges_launch (synchronises); raises as the reference does for an empty window."""
    out, status, picks = pending
    if int(status.max()) != 0:
        raise ValueError("attempt to get argmax of an empty sequence (no velocity inside a ridge window)")
    return (out.cpu().numpy(), picks.cpu().numpy()) if picks is not None else out.cpu().numpy()


def ridges_launch(fv, freqs, vels, freq_lb, freq_ub, ref_freq_idx=None, sigma=25, vel_max=400, ref_vel=None,
                  return_picks=False):
    """The dvh_ridge launch of ridges() without the synchronising read-back: (out, status, picks) device
    tensors for ridges_finish, so that several modes' walks are queued before one wait."""
    if not isinstance(fv, torch.Tensor) or not fv.is_cuda or fv.dtype != torch.float32 or fv.dim() != 3:
        raise ValueError("fv must be a float32 device tensor [B, Nvel, Nfreq] (no CPU fallback)")
    freqs = np.asarray(freqs, dtype=np.float64)
    vel_desc = np.asarray(vels, dtype=np.float64)[::-1].copy()
    fv = fv.contiguous()  # rows [Nvel][Nfreq] as the kernel indexes them
    if vel_desc.size != fv.shape[1] or freqs.size != fv.shape[2]:
        raise ValueError("fv shape does not match (vels, freqs)")
    if vel_desc.size > 1 and not np.all(np.diff(vel_desc) < 0):
        raise ValueError("the device ridge walk needs strictly increasing vels")
    band = np.flatnonzero((freqs >= freq_lb) & (freqs < freq_ub))
    if band.size == 0:
        raise ValueError("empty frequency band")
    if not np.array_equal(band, np.arange(band[0], band[-1] + 1)):
        raise ValueError("the frequency band must be contiguous")
    c0, nb = int(band[0]), int(band.size)
    dev = fv.device
    from .device import upload
    vr = None
    if ref_freq_idx is not None and ref_vel is not None:
        vr = ref_vel(freqs[band]) if callable(ref_vel) else np.asarray(ref_vel, dtype=np.float64)
        vr = np.asarray(vr, dtype=np.float64).reshape(nb)
    # ref_freq_idx=None -> vel_max mode (INT32_MIN); a negative index is a Python index into the band,
    # walked in the reference's loop order (modules/utils.py:662-671)
    ref = -2 ** 31 if ref_freq_idx is None else int(ref_freq_idx)
    if ref_freq_idx is not None and not -nb <= ref < nb:
        raise IndexError(f"index {ref} is out of bounds for axis 0 with size {nb}")
    B = fv.shape[0]
    out = torch.empty((B, nb), dtype=torch.float64, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    # the walk's host tables in one asynchronous copy: the launch is queued without waiting for the work before it
    tabs = upload([vel_desc, np.asarray(_sg_ridge(), dtype=np.float64)] + ([vr] if vr is not None else []), dev)
    vel_t, sg = tabs[0], tabs[1]
    vref = tabs[2] if vr is not None else None
    picks = torch.empty((B, nb), dtype=torch.float64, device=dev) if return_picks else None
    _lib.call("dvh_ridge", _lib.ptr(fv), fv.stride(0), B, fv.shape[1], fv.shape[2], c0, nb, _lib.ptr(vel_t), ref,
              float(sigma), float(vel_max), _lib.ptr(vref), _lib.ptr(sg), 25, _lib.ptr(out), _lib.ptr(status),
              _lib.ptr(picks), _lib.stream_of(dev))
    return out, status, picks


_DISP_PLANS = {}  # (nch, w, dt, freqs, vels) -> DispPlan, shared by GatherCache instances
_STREAMS = {}


def _side_stream(device, k):
    """The k-th side stream of a device (created once)."""
    key = (str(device), k)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(device=device)
    return _STREAMS[key]


class GatherCache:
    """Per-pass gathers [n, R, W] of a window list on the device, computed once
    (VirtualShotGathersFromWindows.get_images' per-pass images: norm=False, two-sided).

    Windows whose time steps round to different lag lengths w (499 / 500 on real axes) share the cache: every
    gather sits zero-padded to the widest W, so that a resample's sum over the padded rows is the reference's
    sum(images) -- VirtualShotGather.__add__ adds the other images' first min(w) lags to the first image's
    (apis/virtual_shot_gather.py:195-199) -- on the first drawn pass's lag axis, whose width and time step its
    dispersion image then takes (compute_disp_image, :247-258)."""

    def __init__(self, windows, pivot, start_x, end_x, wlen=2, include_other_side=True, device=None):
        self.device = device or default_device()
        self.prm = VsgParams(pivot=pivot, start_x=start_x, end_x=end_x, wlen=wlen, norm=False,
                             include_other_side=include_other_side)
        geoms = [pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, self.prm) for w in windows]
        shapes = {tuple(np.shape(w.data)) for w in windows}
        if len(shapes) != 1:
            raise ValueError("bootstrap windows must share one shape")
        n_ch, n_t = shapes.pop()
        self.w_of = np.array([g.w for g in geoms], dtype=np.int64)
        by_w = {}
        for i, g in enumerate(geoms):
            by_w.setdefault(g.w, []).append(i)
        if len(by_w) == 1:
            self.plan = VsgPlan(geoms, self.prm, n_ch, n_t)
            self.G = vsg_gathers(to_device_f32([w.data for w in windows], self.device), self.plan)  # [n, R, w]
        else:
            plans = {w: VsgPlan([geoms[i] for i in idx], self.prm, n_ch, n_t) for w, idx in by_w.items()}
            if len({p.R for p in plans.values()}) != 1:
                raise ValueError("operands could not be broadcast together: passes produce gathers of different shapes")
            self.plan = plans[geoms[0].w]
            W = max(by_w)
            self.G = torch.zeros((len(windows), self.plan.R, W), dtype=torch.float32, device=self.device)
            for w, idx in by_w.items():
                g = vsg_gathers(to_device_f32([windows[i].data for i in idx], self.device), plans[w])
                self.G[torch.as_tensor(idx, device=self.device), :, :w] = g
        self.W = int(self.G.shape[-1])
        self.gx, self.gt = geoms[0].gather_x_axis, geoms[0].gather_t_axis
        # per lag length: the time axis of its first pass (a resample's image takes its first drawn pass's)
        self._gt_of = {}
        for g in geoms:
            self._gt_of.setdefault(g.w, g.gather_t_axis)
        self.n = len(windows)
        self._disp = {}

    @classmethod
    def from_device(cls, data, x_axis, t_axis, trk_x, trk_t, trk_len, pivot, start_x, end_x, wlen=2,
                    include_other_side=True):
        """The cache of windows already resident as one float32 device tensor [n, C, T] on shared axes, with
        the index tables derived on the device from packed trajectories (plan.pack_trajectories layout,
        dvh_pass_geometry): no per-pass host work (the bench's bootstrap job)."""
        from .plan import DevicePlan
        self = cls.__new__(cls)
        self.device = data.device
        self.prm = VsgParams(pivot=pivot, start_x=start_x, end_x=end_x, wlen=wlen, norm=False,
                             include_other_side=include_other_side)
        self.plan = DevicePlan(x_axis, t_axis, trk_x, trk_t, trk_len, self.prm, data.shape[1])
        self.G = vsg_gathers(data, self.plan)
        x_axis, t_axis = np.asarray(x_axis, dtype=np.float64), np.asarray(t_axis, dtype=np.float64)
        pv, st = int(np.argmax(x_axis >= pivot)), int(np.argmax(x_axis >= start_x))
        dt = t_axis[1] - t_axis[0]
        self.gx = x_axis[st:st + self.plan.R] - x_axis[pv]
        self.gt = (np.arange(self.plan.w) - self.plan.w // 2) * dt
        self.n = data.shape[0]
        self.w_of = np.full(self.n, self.plan.w, dtype=np.int64)
        self.W = self.plan.w
        self._gt_of = {self.plan.w: self.gt}
        self._disp = {}
        return self

    def disp_plan(self, start_x=-150, end_x=0, freqs=FREQS, vels=VELS, w=None):
        """compute_disp_image's nearest-offset channel slice and its DispPlan (dx = 8.16, :247-258) for the images
        of lag length w (default: the first pass's)."""
        w = int(self.w_of[0]) if w is None else int(w)
        s = int(np.abs(self.gx - start_x).argmin())
        e = int(np.abs(self.gx - end_x).argmin())
        key = (s, e, id(freqs), id(vels), w)
        if key not in self._disp:
            gt = self._gt_of[w]
            dt = float(gt[1] - gt[0])
            # plans are shared across caches of one geometry (a convergence test per class builds a new cache;
            # the plan's host tables and their device copies are the same)
            pkey = (e + 1 - s, w, dt, np.asarray(freqs, dtype=np.float64).tobytes(),
                    np.asarray(vels, dtype=np.float64).tobytes())
            if pkey not in _DISP_PLANS:
                if len(_DISP_PLANS) >= 16:
                    _DISP_PLANS.pop(next(iter(_DISP_PLANS)))
                _DISP_PLANS[pkey] = DispPlan(e + 1 - s, w, 8.16, dt, freqs, vels)
            self._disp[key] = (s, e, _DISP_PLANS[pkey])
        return self._disp[key]

    def images_of(self, stacks, first, start_x=-150, end_x=0):
        """f-v images [B, Nvel, Nfreq] of resample stacks [B, nch, W] whose first drawn passes are ``first``: each
        on its first pass's lag axis (its width w and time step)."""
        wf = self.w_of[np.asarray(first, dtype=np.int64)]
        if np.all(wf == self.W):
            _, _, plan = self.disp_plan(start_x, end_x, w=self.W)
            return fv_from_fk(fk_grid(stacks, plan), plan)
        out = None
        for w in np.unique(wf):
            rows = np.flatnonzero(wf == w)
            _, _, plan = self.disp_plan(start_x, end_x, w=int(w))
            rt = torch.as_tensor(rows, device=self.device)
            fv = fv_from_fk(fk_grid(stacks[rt][:, :, :int(w)], plan), plan)
            if out is None:
                out = torch.empty((stacks.shape[0],) + tuple(fv.shape[1:]), dtype=fv.dtype, device=fv.device)
            out[rt] = fv
        return out

    def resample_stacks(self, sel, start_x=-150, end_x=0, out=None):
        """Mean gathers over the disp rows for every draw: sel [B, k] pass indices -> [B, nch, w] (into
        ``out``, a contiguous [B, nch, w] float32 device tensor, when given)."""
        sel = np.asarray(sel, dtype=np.int32)
        if sel.ndim != 2 or sel.size == 0 or sel.min() < 0 or sel.max() >= self.n:
            raise ValueError("selections must be [B, k] pass indices")
        s, e, _ = self.disp_plan(start_x, end_x)
        w, R = self.W, self.plan.R
        B, k = sel.shape
        if out is None:
            out = torch.empty((B, e + 1 - s, w), dtype=torch.float32, device=self.device)
        elif tuple(out.shape) != (B, e + 1 - s, w) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous float32 [{B}, {e + 1 - s}, {w}] tensor")
        sel_t = torch.as_tensor(sel, device=self.device)
        base = self.G[:, s:e + 1, :]
        _lib.call("dvh_select_mean", _lib.ptr(base), R * w, (e + 1 - s) * w, _lib.ptr(sel_t), B, k, _lib.ptr(out),
                  (e + 1 - s) * w, _lib.stream_of(self.device))
        return out

    def resample_stacks_sizes(self, sels, start_x=-150, end_x=0, out=None):
        """resample_stacks of several draw sets (sels: list of [B_k, k] arrays, e.g. one per bootstrap size) into
        consecutive rows of one [sum B_k, nch, w] buffer: every selection, with each resample's offset and size,
        crosses to the device in ONE asynchronous copy (device.upload) and all resamples are one
        dvh_select_mean_var launch (60 launches of 30 resamples each were latency-bound: 0.94 ms)."""
        from .device import upload
        sels = [np.asarray(x, dtype=np.int32) for x in sels]
        if not sels or any(x.ndim != 2 or x.size == 0 for x in sels):
            raise ValueError("selections must be [B, k] pass indices")
        flat = np.concatenate([x.reshape(-1) for x in sels])
        if flat.min() < 0 or flat.max() >= self.n:
            raise ValueError("selections must be [B, k] pass indices")
        s, e, _ = self.disp_plan(start_x, end_x)
        w, R = self.W, self.plan.R
        B = sum(x.shape[0] for x in sels)
        rows = (e + 1 - s) * w
        if out is None:
            out = torch.empty((B, e + 1 - s, w), dtype=torch.float32, device=self.device)
        elif tuple(out.shape) != (B, e + 1 - s, w) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous float32 [{B}, {e + 1 - s}, {w}] tensor")
        cnt = np.concatenate([np.full(x.shape[0], x.shape[1], dtype=np.int32) for x in sels])
        off = np.concatenate([[0], np.cumsum(cnt[:-1], dtype=np.int64)]).astype(np.int32)
        sel_t, off_t, cnt_t = upload([flat, off, cnt], self.device)
        base = self.G[:, s:e + 1, :]
        _lib.call("dvh_select_mean_var", _lib.ptr(base), R * w, rows, _lib.ptr(sel_t), _lib.ptr(off_t), _lib.ptr(cnt_t),
                  B, _lib.ptr(out), rows, _lib.stream_of(self.device))
        return out

    def resample_images(self, sel, start_x=-150, end_x=0):
        """f-v images [B, Nvel, Nfreq] of every draw's stack (compute_disp_image(end_x, start_x))."""
        sel = np.asarray(sel, dtype=np.int32)
        return self.images_of(self.resample_stacks(sel, start_x, end_x), sel[:, 0], start_x, end_x)


def bootstrap_ridges(cache: GatherCache, sels, sigma, ref_freq_idx, freq_lb, freq_up, ref_vel, start_x=-150,
                     end_x=0):
    """Ridge velocities per mode for draws ``sels`` [B, k]: list over modes of [B, n_band] arrays."""
    fv = cache.resample_images(sels, start_x, end_x)
    out = []
    for m in range(len(freq_lb)):
        ref = ref_freq_idx[m] - int(np.sum(FREQS < freq_lb[m]))
        out.append(ridges(fv, FREQS, VELS, freq_lb[m], freq_up[m], ref_freq_idx=ref, sigma=sigma[m], vel_max=800,
                          ref_vel=ref_vel[m]))
    return out


def convergence(cache: GatherCache, max_size, bt_times, sigma, ref_freq_idx, freq_lb, freq_up, ref_vel, start_x=-150,
                end_x=0, rand=random, phases=None):
    """The notebooks' convergence_test (imaging_diff_speed.ipynb#cell30) on a gather cache: for bt_size =
    1..max_size, bt_times resamples (the same random.sample draws in the same order as the notebook's
    per-size bootstrap_disp calls), their ridges per mode, and the summed per-frequency std -> [n_modes,
    max_size].  All max_size x bt_times resamples go through ONE dispersion batch (select_mean per size
    into one buffer, one tdft / fk / f-v launch each, one ridge launch per mode), so the host synchronises
    once per mode instead of once per (size, mode).  ``phases`` (optional dict) receives torch events
    around the resample / dispersion / ridge parts for timing."""
    t_draw = time.perf_counter()
    sels = draw_sizes(cache.n, range(1, max_size + 1), bt_times, rand)
    if phases is not None:
        phases["draw_host_s"] = time.perf_counter() - t_draw
    B = max_size * bt_times
    ev = (lambda name: phases.setdefault(name, torch.cuda.Event(enable_timing=True)).record()) if phases is not None \
        else (lambda name: None)
    ev("select0")
    stacks = cache.resample_stacks_sizes(sels, start_x, end_x)
    ev("select1")
    fv = cache.images_of(stacks, np.concatenate([x[:, 0] for x in sels]), start_x, end_x)
    ev("disp1")
    out = np.empty((len(freq_lb), max_size))
    # every mode's walk queued at once, each on its own stream: one walk is one wave per resample (1 800 waves,
    # a fraction of the chip), so the modes run side by side; one wait below
    main = torch.cuda.current_stream(cache.device)
    ready = torch.cuda.Event()
    ready.record(main)
    pend = []
    for m in range(len(freq_lb)):
        st = _side_stream(cache.device, m)
        st.wait_event(ready)
        with torch.cuda.stream(st):
            pend.append(ridges_launch(fv, FREQS, VELS, freq_lb[m], freq_up[m], ref_freq_idx=ref_freq_idx[m] -
                                      int(np.sum(FREQS < freq_lb[m])), sigma=sigma[m], vel_max=800,
                                      ref_vel=ref_vel[m]))
            for t in pend[-1]:
                if t is not None:
                    t.record_stream(main)
        fv.record_stream(st)
        main.wait_stream(st)
    ev("ridge1")
    for m, pd in enumerate(pend):
        r = np.asarray(ridges_finish(pd))
        # per size: the std over its bt_times resamples of each frequency's pick, summed over frequencies
        out[m] = np.std(r.reshape(max_size, bt_times, -1), axis=1).sum(axis=1)
    return out


def draw(n, bt_size, bt_times, rand=random):
    """The reference's draws: bt_times x random.sample(range(1, n), bt_size), bit for bit, formed by the
    library's host routine from the generator's Mersenne Twister state (dvh_random_sample), which is handed
    back so that ``rand`` continues exactly as after Python's own calls.  ``rand``: the ``random`` module or a
    random.Random instance."""
    return draw_sizes(n, [bt_size], bt_times, rand)[0]


def draw_sizes(n, sizes, bt_times, rand=random):
    """[draw(n, k, bt_times, rand) for k in sizes] with one read and one write-back of the generator state."""
    for k in sizes:
        if not 0 <= k <= max(n - 1, 0):
            raise ValueError("Sample larger than population or is negative")
    version, mt, gauss = rand.getstate()
    st = np.array(mt, dtype=np.uint32)
    outs = []
    for k in sizes:
        out = np.empty((bt_times, k), dtype=np.int64)
        _lib.call("dvh_random_sample", st.ctypes.data, 1, max(n - 1, 0), k, bt_times, out.ctypes.data)
        outs.append(out.astype(np.int32))
    rand.setstate((version, tuple(int(v) for v in st), gauss))
    return outs


def save_ridge_npz(file_name, freqs, freq_lb, freq_ub, reference_layout=False, **ridges):
    """The ridge-statistics npz of the notebooks (imaging_diff_speed.ipynb#cell27, data/<x0>_speeds.npz:
    ``freqs, freq_lb, freq_ub, vels_<class>``) for bootstrap_disp results.  ``ridges``: class name ->
    ridge_vel, bootstrap_disp's list over modes of per-resample ridge arrays (modes have different band
    lengths).  By default the file is pickle-free: ``vels_<class>`` is omitted and each mode is a dense
    ``vels_<class>_m<k>`` [n_resample, n_band_k] array (load with allow_pickle=False, load_ridge_npz).
    reference_layout=True writes ``vels_<class>`` as the notebook's ragged object array instead (np.savez
    pickles it; only the notebook's own np.load(allow_pickle=True) reads that)."""
    out = dict(freqs=np.asarray(freqs, dtype=np.float64), freq_lb=np.asarray(freq_lb),
               freq_ub=np.asarray(freq_ub))
    for name, per_mode in ridges.items():
        if reference_layout:
            arr = np.empty(len(per_mode), dtype=object)
            for k, rv in enumerate(per_mode):
                arr[k] = list(rv)
            out[f"vels_{name}"] = arr
        else:
            for k, rv in enumerate(per_mode):
                out[f"vels_{name}_m{k}"] = np.asarray(rv, dtype=np.float64).reshape(len(rv), -1)
    np.savez(file_name, **out)


def load_ridge_npz(file_name):
    """(freqs, freq_lb, freq_ub, {class: [per-mode [n_resample, n_band] arrays]}) of a pickle-free
    save_ridge_npz file (allow_pickle=False)."""
    with np.load(file_name, allow_pickle=False) as f:
        ridges = {}
        for key in sorted(k for k in f.files if k.startswith("vels_")):
            name, _, m = key[5:].rpartition("_m")
            ridges.setdefault(name, {})[int(m)] = f[key]
        return (f["freqs"], f["freq_lb"], f["freq_ub"],
                {n: [d[k] for k in sorted(d)] for n, d in ridges.items()})
