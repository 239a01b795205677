"""Per-pass windowing / taper / bandpass on device (host side builds the small index tables).

  bandpass_inplace  bandpass_data (modules/utils.py:179-189): butter(10, [flo, fhi] / fNy, 'band',
                    output='sos') designed on the host (filter design, 10 x 6 coefficients), the
                    zero-phase filtering itself in dvh_sosfiltfilt
  mute_along_traj   apis/data_classes.py:49-72: per time sample the taper placement
                    (argmax(x > car(t) - offset/2 + delta_x), clipped) is tabulated on the host with
                    the reference's float64 expressions; the multiply runs in dvh_mute_traj
  mute_along_time   apis/data_classes.py:100-104 -> dvh_mute_time
  surface_wave_preprocessing  TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:
                    51-71): bandpass + empty / noisy trace imputation + per-trace L2 norm
"""
from __future__ import annotations

import numpy as np
import scipy.signal
import torch

from . import _lib
from .device import default_device
from .plan import interp1d_extrap


def butter_bandpass_sos(dt, flo, fhi, order=10):
    fny = 0.5 / dt
    return scipy.signal.butter(order, [flo / fny, fhi / fny], analog=False, btype="band", output="sos")


def _padlen(sos):
    return 3 * (2 * len(sos) + 1 - min(int((sos[:, 2] == 0).sum()), int((sos[:, 5] == 0).sum())))


def tukey(n, alpha):
    """scipy.signal.windows.tukey(n, alpha) (sym=True)."""
    return scipy.signal.windows.tukey(n, alpha)


class _DeviceView:
    """Device tensor for a host array or tensor, written back in place on exit."""

    def __init__(self, data):
        self.data = data
        if isinstance(data, torch.Tensor) and data.is_cuda:
            self.t = data if data.is_contiguous() else data.contiguous()
        else:
            host = np.asarray(data.detach().cpu() if isinstance(data, torch.Tensor) else data)
            if host.dtype not in (np.float32, np.float64):
                raise TypeError("data must be float32 or float64")
            self.t = torch.from_numpy(np.ascontiguousarray(host)).to(default_device())
        if self.t.dtype not in (torch.float32, torch.float64):
            raise TypeError("data must be float32 or float64")
        self.dtype = 0 if self.t.dtype == torch.float32 else 1

    def write_back(self):
        d = self.data
        if isinstance(d, torch.Tensor):
            if d.data_ptr() != self.t.data_ptr():
                d.copy_(self.t)
        else:
            d[...] = self.t.to("cpu").numpy()


_DESIGNS = {}


def _design(dt, flo, fhi, dev):
    """(sos, zi, padlen) of bandpass_data's filter and their device copies, cached per (dt, band, device):
    the design is a pure function of its arguments (the reference redesigns it per call)."""
    key = (float(dt), float(flo), float(fhi), str(dev))
    if key not in _DESIGNS:
        sos = butter_bandpass_sos(dt, flo, fhi)
        zi = scipy.signal.sosfilt_zi(sos)
        _DESIGNS[key] = (sos, _padlen(sos), torch.from_numpy(np.ascontiguousarray(sos, dtype=np.float64)).to(dev),
                         torch.from_numpy(np.ascontiguousarray(zi, dtype=np.float64)).to(dev))
    return _DESIGNS[key]


_PLANS = {}
SOS_MFMA_MAX_POLE = 0.999  # include/dvh.h DVH_SOS_MFMA_MAX_POLE


def _plan(key, n_t, sos, padlen, sos_t, zi_t, dev):
    """dvh_sosfiltfilt_plan's block operators of the design, per record length (formed once; the reference
    redesigns the same filter for every record); None (the block recursion) for a design whose largest pole
    radius exceeds SOS_MFMA_MAX_POLE, where the matrix form's rounding would pass 1e-10 of the output."""
    k = key + (int(n_t),)
    if k not in _PLANS:
        s64 = np.ascontiguousarray(sos, dtype=np.float64)
        if _lib.load().dvh_sos_pole_radius(s64.ctypes.data, len(sos)) > SOS_MFMA_MAX_POLE:
            _PLANS[k] = None
            return None
        plan = torch.empty(int(_lib.load().dvh_sosfiltfilt_plan_bytes(len(sos))) // 8, dtype=torch.float64, device=dev)
        _lib.call("dvh_sosfiltfilt_plan", _lib.ptr(sos_t), len(sos), _lib.ptr(zi_t), int(n_t), padlen, _lib.ptr(plan),
                  _lib.stream_of(dev))
        _PLANS[k] = plan
    return _PLANS[k]


def bandpass_inplace(data, dt, flo, fhi):
    v = _DeviceView(data)
    t = v.t
    n_t = t.shape[-1]
    rows = t.reshape(-1, n_t)
    dev = t.device
    sos, padlen, sos_t, zi_t = _design(dt, flo, fhi, dev)
    if n_t <= padlen:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {padlen}.")
    nbytes = int(_lib.load().dvh_sosfiltfilt_workspace(rows.shape[0], n_t, len(sos), padlen))
    work = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=dev)
    plan = _plan((float(dt), float(flo), float(fhi), str(dev)), n_t, sos, padlen, sos_t, zi_t, dev)
    _lib.call("dvh_sosfiltfilt_planned", _lib.ptr(rows), v.dtype, rows.shape[0], rows.stride(0), n_t, _lib.ptr(sos_t),
              len(sos), padlen, _lib.ptr(zi_t), None if plan is None else _lib.ptr(plan), _lib.ptr(work),
              _lib.stream_of(dev))
    v.write_back()
    return data


def mute_traj_table(x_axis, t_axis, veh_state_x, veh_state_t, offset=200, alpha=0.3, delta_x=20):
    """[T, 3] = (start, end, taper_start) per time sample and the taper, as the reference places them."""
    f = interp1d_extrap(veh_state_t, veh_state_x)
    car = f(np.asarray(t_axis, dtype=np.float64))
    x_axis = np.asarray(x_axis, dtype=np.float64)
    dx = x_axis[1] - x_axis[0]
    nx = x_axis.size
    n_samp = int(offset / dx)
    center = car - offset / 2 + delta_x
    c = np.argmax(x_axis[None, :] > center[:, None], axis=1)
    s = np.maximum(0, c - n_samp // 2)
    e = np.minimum(nx, c + n_samp // 2)
    ts = s + n_samp // 2 - c
    return np.stack([s, e, ts], axis=1).astype(np.int32), tukey(n_samp, alpha)


def mute_along_traj(window, offset=200, alpha=0.3, delta_x=20):
    tab, taper = mute_traj_table(window.x_axis, window.t_axis, window.veh_state_x, window.veh_state_t, offset, alpha,
                                 delta_x)
    v = _DeviceView(window.data)
    n_ch, n_t = v.t.shape[-2], v.t.shape[-1]
    dev = v.t.device
    tab_t = torch.from_numpy(np.ascontiguousarray(tab)).to(dev)
    taper_t = torch.from_numpy(np.ascontiguousarray(taper, dtype=np.float64)).to(dev)
    _lib.call("dvh_mute_traj", _lib.ptr(v.t), v.dtype, 1, n_ch * n_t, n_ch, n_t, _lib.ptr(tab_t), _lib.ptr(taper_t),
              _lib.stream_of(dev))
    v.write_back()


def mute_along_time(window, alpha=0.3):
    v = _DeviceView(window.data)
    n_t = v.t.shape[-1]
    dev = v.t.device
    taper_t = torch.from_numpy(np.ascontiguousarray(tukey(n_t, alpha), dtype=np.float64)).to(dev)
    _lib.call("dvh_mute_time", _lib.ptr(v.t), v.dtype, v.t.numel() // n_t, n_t, _lib.ptr(taper_t),
              _lib.stream_of(dev))
    v.write_back()


def surface_wave_preprocessing(data, dt, method="surface_wave", flo=1.2, fhi=30, impute_noise_traces=True,
                               noise_threshold=5, impute_empty_traces=True, return_indices=False, _phases=None):
    """TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71) of a
    continuous record [n_ch, n_t] -> ``data_for_imaging`` (a new array; the input is left as is):
    bandpass_data(flo, fhi) (dvh_sosfiltfilt), then find_noise_idx / impute_noisy_trace for an empty
    trace and for a noisy trace, then for method 'surface_wave' the per-trace L2 norm
    (dvh_trace_cleanup).  Host arrays in -> host arrays out in the record's dtype, like the
    reference's data.copy(): a float32 record is filtered in float64 and stored in float32, then
    imputed and normalised in float32 (other dtypes are imaged as float64); device tensors stay on the
    device.  With return_indices, also the (empty, noisy) trace indices imputed."""
    if method not in ("surface_wave", "xcorr"):
        raise AssertionError("method must be 'surface_wave' or 'xcorr'")
    on_device = isinstance(data, torch.Tensor) and data.is_cuda
    if on_device:
        t = data.clone()
    else:
        host = np.asarray(data.detach().cpu() if isinstance(data, torch.Tensor) else data)
        dt_keep = np.float32 if host.dtype == np.float32 else np.float64
        t = torch.from_numpy(np.array(host, dtype=dt_keep, copy=True)).to(default_device())
    if t.dim() != 2:
        raise ValueError("data must be [n_ch, n_t]")
    ev = (lambda k: _phases.setdefault(k, torch.cuda.Event(enable_timing=True)).record()) if _phases is not None \
        else (lambda k: None)  # timing hook (bench.py --workload prep)
    ev("bandpass0")
    bandpass_inplace(t, dt, flo, fhi)
    ev("bandpass1")
    dev = t.device
    stats = torch.empty(2 * t.shape[0], dtype=torch.float64, device=dev)
    idx = torch.zeros(2, dtype=torch.int32, device=dev)
    flags = (1 if impute_empty_traces else 0) | (2 if impute_noise_traces else 0) | (4 if method == "surface_wave" else 0)
    _lib.call("dvh_trace_cleanup", _lib.ptr(t), 0 if t.dtype == torch.float32 else 1, t.shape[0], t.stride(0),
              t.shape[1], flags, float(noise_threshold), _lib.ptr(stats), _lib.ptr(idx), _lib.stream_of(dev))
    ev("cleanup1")
    out = t if on_device else t.cpu().numpy()
    if return_indices:
        return out, tuple(int(i) for i in idx.cpu())
    return out
