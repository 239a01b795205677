"""Hot-path functions of modules/utils.py of the reference, served by the HIP kernels.

  fk            modules/utils.py:236-248  -> full |FK| grid from the dispersion GEMMs
  map_fv        modules/utils.py:457-475  -> dvh_disp_tdft / dvh_disp_fk / dvh_disp_fv
  Dispersion    modules/utils.py:383-426  (same constructor, attributes, npz format, arithmetic)
  bandpass_data modules/utils.py:179-189  -> dvh_sosfiltfilt (zero-phase order-10 Butterworth)
  extract_ridge_ref_idx modules/utils.py:621-678 -> dvh_ridge (one wave per ridge)
  disp_curve_stats  the statistics of plot_disp_curves (:680-713), without the figure
Host arrays in, host arrays out, like the reference; device tensors are accepted too.
"""
from __future__ import annotations

import copy
import os

import numpy as np
import torch

from ..device import default_device


def _as_device_batch(data, device=None):
    device = device or default_device()
    if isinstance(data, torch.Tensor):
        t = data.to(device=device, dtype=torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(data, dtype=np.float32))).to(device)
    if t.dim() == 2:
        t = t.unsqueeze(0)
    return t.contiguous() if t.stride(-1) != 1 else t


_PLANS = {}


def disp_plan(nch, nt, dx, dt, freqs, vels, full_grid=False):
    from ..disp import DispPlan
    freqs = np.asarray(freqs, dtype=np.float64)
    vels = np.asarray(vels, dtype=np.float64)
    key = (nch, nt, float(dx), float(dt), freqs.tobytes(), vels.tobytes(), full_grid)
    if key not in _PLANS:
        if len(_PLANS) > 64:
            _PLANS.clear()
        _PLANS[key] = DispPlan(nch, nt, dx, dt, freqs, vels, full_grid=full_grid)
    return _PLANS[key]


def fk(data, dx, dt):
    """|fftshift(fft2(data, s=[nk, nf]))|, fft_f, fft_k (float32 magnitudes from the MFMA GEMMs)."""
    from ..disp import fk_grid
    t = _as_device_batch(data)
    nch, nt = t.shape[1], t.shape[2]
    plan = disp_plan(nch, nt, dx, dt, [1.0] * 25, [1.0], full_grid=True)
    g = fk_grid(t, plan)[0].to("cpu").numpy()
    return g, plan.fft_f, plan.fft_k


def map_fv(data, dx, dt, freqs, vels, norm=False):
    """f-v image [Nvel, Nfreq] (float32, rows in sorted-query order like interp2d)."""
    from ..disp import fv_maps
    t = _as_device_batch(data)
    plan = disp_plan(t.shape[1], t.shape[2], dx, dt, freqs, vels)
    return fv_maps(t, plan, norm=norm)[0].to("cpu").numpy()


class Dispersion:
    def __init__(self, data, dx, dt, freqs, vels, norm=False, compute_fv=True):
        self.data = data
        self.dx = dx
        self.dt = dt
        self.freqs = freqs
        self.vels = vels
        self.norm = norm
        if compute_fv:
            self._map_fv()

    def save_to_npz(self, fname, fdir="./"):
        np.savez(os.path.join(fdir, fname), freqs=self.freqs, vels=self.vels, fv_map=self.fv_map)

    @classmethod
    def get_dispersion_obj(cls, fname, fdir="./"):
        f = np.load(os.path.join(fdir, fname), allow_pickle=False)
        obj = Dispersion(data=None, dx=None, dt=None, freqs=f["freqs"], vels=f["vels"], compute_fv=False)
        obj.fv_map = f["fv_map"]
        return obj

    def _map_fv(self):
        self.fv_map = map_fv(self.data, self.dx, self.dt, freqs=self.freqs, vels=self.vels, norm=self.norm)

    def plot_image(self, *args, **kwargs):
        raise NotImplementedError("plotting is outside the accelerated path; use the reference's plot_fv_map on "
                                  "obj.fv_map / obj.freqs / obj.vels")

    def __add__(self, other):
        sum_ = Dispersion(self.data, self.dx, self.dt, self.freqs, self.vels, compute_fv=False)
        sum_.fv_map = self.fv_map + other.fv_map
        return sum_

    def __radd__(self, other):
        if other == 0:
            return self
        return self.__add__(other)

    def __truediv__(self, other):
        div_ = copy.deepcopy(self)
        div_.fv_map /= other
        return div_


def bandpass_data(data, dt, flo, fhi):
    """In-place zero-phase Butterworth bandpass (order 10, SOS) along time, on device."""
    from ..preprocess import bandpass_inplace
    bandpass_inplace(data, dt, flo, fhi)


def extract_ridge_ref_idx(freq, vel, fv_map, ref_freq_idx=None, sigma=25, vel_max=400, ref_vel=None):
    """modules/utils.py:621-678 (fv_map [Nvel, Nfreq] with rows in vel[::-1] order), walked on the
    device by dvh_ridge (das_diff_veh_amd.bootstrap.ridges)."""
    import torch

    from ..bootstrap import ridges
    fv = torch.as_tensor(np.ascontiguousarray(fv_map, dtype=np.float32), device=default_device())[None]
    freq = np.asarray(freq, dtype=np.float64)
    out = ridges(fv, freq, vel, freq[0], np.nextafter(freq[-1], np.inf), ref_freq_idx=ref_freq_idx, sigma=sigma,
                 vel_max=vel_max, ref_vel=ref_vel)[0]
    return out


def disp_curve_stats(freqs, freq_lb, freq_up, ridge_vels):
    """The statistics of plot_disp_curves (modules/utils.py:680-713) without the figure:
    per mode the mean, range (max - min) and std over resamples of the ridge velocities."""
    means, ranges, stds = [], [], []
    for i in range(len(ridge_vels)):
        rv = np.array([d for d in ridge_vels[i]], dtype=np.float64)
        means.append(np.mean(rv, axis=0))
        stds.append(np.std(rv, axis=0))
        ranges.append(np.max(rv, axis=0) - np.min(rv, axis=0))
    return means, ranges, stds
