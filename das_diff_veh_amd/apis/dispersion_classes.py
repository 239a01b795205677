"""SurfaceWaveDispersion — drop-in for apis/dispersion_classes.py:9-65 of the reference.

Per-pass dispersion image straight from a window ("naive": raw channel slice, :24-32; "smart":
time + trajectory mutes on a copy first, :34-43), with the reference's stacking arithmetic.
``batched_surface_wave_dispersion`` is the batched flavour-B path used by
DispersionImagesFromWindows.get_images: all passes in one launch of each dispersion kernel, the
per-class mean f-v image formed on device.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from ..modules.utils import Dispersion, disp_plan


class SurfaceWaveDispersion:
    def __init__(self, window, freqs=np.arange(0.8, 25, 0.1), vels=np.arange(200, 1200), method="naive", norm=True,
                 **method_kwargs):
        self.window = window
        self.freqs = freqs
        self.vels = vels
        self.method = method
        self.norm = norm
        if method == "naive":
            self._naive_disp(**method_kwargs)
        else:
            self._smart_disp(**method_kwargs)

    def _naive_disp(self, start_x, end_x):
        dist = end_x - start_x
        window = self.window
        dx = window.x_axis[1] - window.x_axis[0]
        s = int(np.argmax(window.x_axis >= start_x))
        nx = int(dist / dx)
        self.disp = Dispersion(window.data[s:s + nx], dx, window.t_axis[1] - window.t_axis[0], freqs=self.freqs,
                               vels=self.vels, norm=self.norm)

    def _smart_disp(self, mute_along_time=True, time_alpha=0.3, mute_along_traj=True):
        w = copy.deepcopy(self.window)
        if mute_along_time and not getattr(w, "muted_along_time", False):
            w.mute_along_time(alpha=time_alpha)
        if mute_along_traj and not getattr(w, "muted_along_traj", False):
            w.mute_along_traj()
        dx = w.x_axis[1] - w.x_axis[0]
        self.disp = Dispersion(w.data, dx, w.t_axis[1] - w.t_axis[0], freqs=self.freqs, vels=self.vels,
                               norm=self.norm)

    def save_to_npz(self, *args, **kwargs):
        self.disp.save_to_npz(*args, **kwargs)

    def plot_image(self, *args, **kwargs):
        self.disp.plot_image(*args, **kwargs)

    def __add__(self, other):
        sum_ = copy.deepcopy(self)
        sum_.disp = self.disp + other.disp
        return sum_

    def __radd__(self, other):
        if other == 0:
            return self
        return self.__add__(other)

    def __truediv__(self, other):
        new_obj = copy.deepcopy(self)
        new_obj.disp = self.disp / other
        return new_obj

    @classmethod
    def _from_fv(cls, window, freqs, vels, method, norm, fv):
        obj = cls.__new__(cls)
        obj.window, obj.freqs, obj.vels, obj.method, obj.norm = window, freqs, vels, method, norm
        obj.disp = Dispersion(None, None, None, freqs, vels, norm=norm, compute_fv=False)
        obj.disp.fv_map = fv
        return obj


def _naive_groups(windows, start_x, end_x):
    """Window indices per (shape, first channel, channels, dx, dt) of _naive_disp (:24-32)."""
    groups = {}
    for i, w in enumerate(windows):
        dx = w.x_axis[1] - w.x_axis[0]
        s = int(np.argmax(w.x_axis >= start_x))
        nx = int((end_x - start_x) / dx)
        key = (tuple(np.shape(w.data)), s, nx, float(dx), float(w.t_axis[1] - w.t_axis[0]))
        groups.setdefault(key, []).append(i)
    return groups


def _device_windows(windows, idx, mute_offset):
    """Same-shape windows ``idx`` as one float32 device batch; with ``mute_offset`` the windows not yet
    muted are muted along their trajectories on the device copy (mute_along_traj(offset) of a deepcopy,
    ImagesFromWindows.get_images apis/imaging_classes.py:100-102; one dvh_mute_traj launch)."""
    from .. import _lib
    from ..device import to_device_f32
    from ..preprocess import mute_traj_table
    data = to_device_f32([windows[i].data for i in idx])
    mute = [k for k, i in enumerate(idx) if mute_offset is not None and not windows[i].muted_along_traj]
    if mute:
        tabs = []
        for k in mute:
            w = windows[idx[k]]
            tab, taper = mute_traj_table(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, offset=mute_offset)
            tabs.append(tab)
        sub = data if len(mute) == len(idx) else data[mute].contiguous()
        dev = sub.device
        tab_t = torch.from_numpy(np.ascontiguousarray(np.stack(tabs))).to(dev)
        taper_t = torch.from_numpy(np.ascontiguousarray(taper, dtype=np.float64)).to(dev)
        _lib.call("dvh_mute_traj", _lib.ptr(sub), 0, len(mute), sub.stride(0), sub.shape[1], sub.shape[2],
                  _lib.ptr(tab_t), _lib.ptr(taper_t), _lib.stream_of(dev))
        if sub is not data:
            data[mute] = sub
    return data


def sharded_dispersion_means(windows, slots=None, n_slot=1, group=None, norm=False, freqs=np.arange(0.8, 25, 0.1),
                             vels=np.arange(200, 1200), start_x=None, end_x=None, mute_offset=None):
    """Flavour B (per-pass f-v maps averaged per class) over the ranks of ``group``: every rank holds the
    same window list and class ``slots``; each images its shard of the passes (distributed.shard_passes)
    as naive dispersion (SurfaceWaveDispersion._naive_disp, apis/dispersion_classes.py:24-32, after the
    trajectory mute of get_images when ``mute_offset`` is set) and sums its passes' |FK| grids per class
    with weights 1 / global class count; ONE all-reduce of [n_slot, n_k, n_f] (float64) and one f-v
    sampling give every rank the class-mean f-v images sum(images) / len(images)
    (apis/imaging_classes.py:106-107, 120-126): the sampling after |FK| is linear.
    Returns (fv [n_slot, Nvel, Nfreq] float32 device tensor, this rank's pass indices)."""
    from ..disp import fk_grid, fv_from_fk
    from ..distributed import sharded_class_means
    slots = np.zeros(len(windows), dtype=np.int64) if slots is None else np.asarray(slots, dtype=np.int64)
    if len(windows) == 0 or slots.shape != (len(windows),):
        raise ValueError("need one class slot per window")
    groups = _naive_groups(windows, start_x, end_x)
    # one plan per f-v input geometry (channels, samples, dx, dt); windows of different geometries give
    # f-v maps of one shape that the reference simply adds, so their |FK| grids travel side by side in
    # one buffer [n_slot, sum of grid sizes] and each is sampled on its own plan after the exchange
    plans, off = {}, 0
    for (shape, _, nx, dx, dt) in groups:
        g = (nx, shape[1], dx, dt)
        if g not in plans:
            plan = disp_plan(*g, freqs, vels)
            plans[g] = (plan, off)
            off += plan.n_kb * plan.n_fb
    from ..device import default_device
    dev = default_device()

    def grid(buf, g):
        plan, o = plans[g]
        return buf[:, o:o + plan.n_kb * plan.n_fb].view(n_slot, plan.n_kb, plan.n_fb)

    def partial(mine, weights):
        buf = torch.zeros((n_slot, off), dtype=torch.float64, device=dev)
        wmap = dict(zip(mine.tolist(), weights.tolist()))
        for (shape, s, nx, dx, dt), idx in groups.items():
            loc = [i for i in idx if i in wmap]
            if loc:
                g = (nx, shape[1], dx, dt)
                data = _device_windows(windows, loc, mute_offset)[:, s:s + nx, :]
                grid(buf, g).add_(fk_grid(data, plans[g][0], norm=norm, slots=slots[loc], weights=[wmap[i] for i in loc],
                                          n_slot=n_slot))
        return buf

    buf, mine = sharded_class_means(partial, slots, n_slot, group)
    fv = None
    for g, (plan, _) in plans.items():
        part = fv_from_fk(grid(buf, g).contiguous(), plan)
        fv = part if fv is None else fv + part
    return fv, mine


def batched_surface_wave_dispersion(windows, norm=False, freqs=np.arange(0.8, 25, 0.1), vels=np.arange(200, 1200),
                                    method="naive", start_x=None, end_x=None, mute_offset=None, **kw):
    """(images, avg_image) of ImagesFromWindows.get_images for image_cls=SurfaceWaveDispersion,
    naive method: one launch per kernel for all windows of a shape.  With ``mute_offset``, every
    window not yet muted is muted along its trajectory first (mute_along_traj(offset=mute_offset) on
    a copy, as get_images does): one dvh_mute_traj launch over the device batch, the windows
    themselves untouched."""
    from ..disp import fk_grid, fv_from_fk
    if method != "naive" or kw:
        if mute_offset is not None:
            windows = [copy.deepcopy(w) if not w.muted_along_traj else w for w in windows]
            for w in windows:
                if not w.muted_along_traj:
                    w.mute_along_traj(offset=mute_offset)
        images = [SurfaceWaveDispersion(w, freqs=freqs, vels=vels, method=method, norm=norm,
                                        **({} if method != "naive" else dict(start_x=start_x, end_x=end_x)), **kw)
                  for w in windows]
        avg = sum(images) / len(images)
        return images, avg
    groups = _naive_groups(windows, start_x, end_x)
    n = len(windows)
    acc = None
    per_pass = [None] * n
    for (shape, s, nx, dx, dt), idx in groups.items():
        data = _device_windows(windows, idx, mute_offset)
        data = data[:, s:s + nx, :]
        plan = disp_plan(data.shape[1], data.shape[2], dx, dt, freqs, vels)
        FK = fk_grid(data, plan, norm=norm)
        fv = fv_from_fk(FK, plan)
        host = fv.to("cpu").numpy()
        for k, i in enumerate(idx):
            per_pass[i] = host[k]
        part = fv.sum(dim=0)
        acc = part if acc is None else acc + part
    images = [SurfaceWaveDispersion._from_fv(w, freqs, vels, method, norm, per_pass[i]) for i, w in enumerate(windows)]
    avg_fv = (acc / n).to("cpu").numpy()
    avg = SurfaceWaveDispersion._from_fv(windows[0], freqs, vels, method, norm, avg_fv)
    return images, avg
