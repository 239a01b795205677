"""VirtualShotGather — drop-in for apis/virtual_shot_gather.py:183-270 of the reference.

The constructor signature, keyword defaults (those of construct_shot_gather, :165-166), attributes
(``XCF_out`` float64 [R, w], ``x_axis``, ``t_axis``, ``disp``, ``window``) and the stacking
arithmetic (``__add__``, ``__radd__(0)``, ``__truediv__``) are the reference's; the correlation
itself runs in the HIP kernels of libdvh (das_diff_veh_amd/csrc/dvh_vsg.hip).  Errors the reference
raises for unusable inputs (the dt == 0.004 window-length mismatch, out-of-order gather geometry)
are raised as ValueError before any launch.
"""
from __future__ import annotations

import copy
import os

import numpy as np

from .. import engine
from ..plan import VsgParams

_POSITIONAL = ("start_x", "end_x", "pivot", "wlen", "norm", "norm_amp", "time_window_to_xcorr", "delta_t")


def vsg_params(include_other_side=False, *args, **kwargs):
    """construct_shot_gather(window, start_x=530, end_x=680, pivot=635, wlen=2, norm=True, norm_amp=True,
    time_window_to_xcorr=4, delta_t=1) keyword surface -> VsgParams."""
    if len(args) > len(_POSITIONAL):
        raise TypeError("too many positional arguments")
    kw = dict(zip(_POSITIONAL, args))
    for k, v in kwargs.items():
        if k in kw:
            raise TypeError(f"got multiple values for argument '{k}'")
        if k not in _POSITIONAL:
            raise TypeError(f"construct_shot_gather() got an unexpected keyword argument '{k}'")
        kw[k] = v
    return VsgParams(include_other_side=bool(include_other_side), **kw)


class VirtualShotGather:
    def __init__(self, window, compute_xcorr=True, disp=None, include_other_side=False, *args, **kwargs):
        self.window = window
        self.disp = disp
        if compute_xcorr:
            prm = vsg_params(include_other_side, *args, **kwargs)
            res, geoms = engine.gathers([window], prm)
            self.XCF_out, self.x_axis, self.t_axis = res[0], geoms[0].gather_x_axis, geoms[0].gather_t_axis

    @classmethod
    def _from_arrays(cls, window, xcf, x_axis, t_axis):
        obj = cls(window=window, compute_xcorr=False)
        obj.XCF_out, obj.x_axis, obj.t_axis = xcf, x_axis, t_axis
        return obj

    def __add__(self, other):
        sum_ = copy.deepcopy(self)
        length = min(self.XCF_out.shape[-1], other.XCF_out.shape[-1])
        sum_.XCF_out[:, :length] += other.XCF_out[:, :length]
        return sum_

    def __radd__(self, other):
        if other == 0:
            return self
        return self.__add__(other)

    def __truediv__(self, other):
        new_obj = copy.deepcopy(self)
        new_obj.XCF_out /= other
        return new_obj

    @classmethod
    def get_VirtualShotGather_obj(cls, fdir, fname):
        new_obj = cls(window=None, compute_xcorr=False)
        f = np.load(os.path.join(fdir, fname), allow_pickle=False)
        new_obj.XCF_out, new_obj.x_axis, new_obj.t_axis = f["XCF_out"], f["x_axis"], f["t_axis"]
        return new_obj

    def save_to_npz(self, fname, fdir, **kwargs):
        np.savez(os.path.join(fdir, fname), XCF_out=self.XCF_out, x_axis=self.x_axis, t_axis=self.t_axis, **kwargs)

    def compute_disp_image(self, freqs=np.arange(0.8, 25, 0.1), vels=np.arange(200, 1200), norm=False,
                           start_x=None, end_x=None):
        """apis/virtual_shot_gather.py:247-258: nearest-offset channel slice -> Dispersion(dx=8.16)."""
        from ..modules.utils import Dispersion
        if start_x is None:
            start_x = self.x_axis[0]
        if end_x is None:
            end_x = self.x_axis[-1]
        s = np.abs(self.x_axis - start_x).argmin()
        e = np.abs(self.x_axis - end_x).argmin()
        self.disp = Dispersion(self.XCF_out[s:e + 1], 8.16, self.t_axis[1] - self.t_axis[0], freqs=freqs, vels=vels,
                               norm=norm)

    def save_disp_to_npz(self, *args, **kwargs):
        assert self.disp, "please run obj.compute_disp_image() first"
        self.disp.save_to_npz(*args, **kwargs)

    def norm(self):
        self.XCF_out /= np.linalg.norm(self.XCF_out, axis=-1, keepdims=True)

    def plot_image(self, *args, **kwargs):
        raise NotImplementedError("plotting is outside the accelerated path; use the reference's plot_xcorr on "
                                  "obj.XCF_out / obj.x_axis / obj.t_axis")

    plot_disp = plot_image
    plot_spec_vs_offset = plot_image
