"""TimeLapseImaging — the imaging half of apis/timeLapseImaging.py:22-211 on the device.

Mirrors the reference class's constructor, attributes and imaging methods:
  _preprocessing_for_surface_waves  :50-71   bandpass + empty / noisy trace imputation + trace norm
                                             (preprocess.surface_wave_preprocessing, dvh_sosfiltfilt,
                                             dvh_trace_cleanup)
  select_surface_wave_windows       :166-196 SurfaceWaveSelector on data_for_imaging (sw_selector)
                                             and on the raw data (qs_selector), cut on the device
  get_images                        :198-201 DispersionImagesFromWindows (flavour B) or
                                             VirtualShotGathersFromWindows (xcorr) of sw_selector
  save_avg_disp_to_npz              :205-206
Vehicle tracking (_preprocess_for_tracking :73-104, track_cars :106-120: KF_tracking of
apis/tracking.py) is outside the device hot path: the constructor skips it and the
tracking results (veh_states on the 1 m / 50 Hz tracking grid) are attached with ``set_tracking``,
e.g. from the reference's own tracker or from stored tracks.
"""
from __future__ import annotations

import numpy as np

from ..preprocess import surface_wave_preprocessing
from .data_classes import SurfaceWaveSelector
from .imaging_classes import DispersionImagesFromWindows, VirtualShotGathersFromWindows

channel_prop = {"odh3": {"start_ch": 400, "dx": 8.16}}  # apis/timeLapseImaging.py:14-19


class TimeLapseImaging:
    def __init__(self, data, x_axis, t_axis, interrogator="odh3", method="surface_wave",
                 tracking_preprecessing_dict=None, surface_wave_preprecessing_dict=None):
        assert method in {"surface_wave", "xcorr"}
        self.method = method
        prop = channel_prop[interrogator]
        self.data = data
        self.t_axis = t_axis
        self.dt = self.t_axis[1] - self.t_axis[0]
        self.x_axis = x_axis
        self.start_ch = prop["start_ch"]
        self.dx = prop["dx"]
        self.distances_along_fiber = (x_axis - self.start_ch) * self.dx
        self.tracking_preprecessing_dict = tracking_preprecessing_dict if tracking_preprecessing_dict is not None else {}
        self.surface_wave_preprecessing_dict = surface_wave_preprecessing_dict
        self._preprocessing_for_surface_waves()

    def _preprocessing_for_surface_waves(self, impute_noise_traces=True, noise_threshold=5, impute_empty_traces=True):
        if self.surface_wave_preprecessing_dict is None:
            self.surface_wave_preprecessing_dict = {}
        flo = self.surface_wave_preprecessing_dict.get("flo", 1.2)
        fhi = self.surface_wave_preprecessing_dict.get("fhi", 30)
        self.data_for_imaging = surface_wave_preprocessing(
            self.data, self.dt, method=self.method, flo=flo, fhi=fhi, impute_noise_traces=impute_noise_traces,
            noise_threshold=noise_threshold, impute_empty_traces=impute_empty_traces)

    def set_tracking(self, veh_states, start_x, dist_along_fiber_tracking, t_axis_tracking, end_x=None):
        """The attributes track_cars / _preprocess_for_tracking leave behind (:73-120)."""
        self.veh_states = np.asarray(veh_states)
        self.start_x = start_x
        self.end_x = end_x
        self.dist_along_fiber_tracking = np.asarray(dist_along_fiber_tracking)
        self.t_axis_tracking = np.asarray(t_axis_tracking)

    def track_cars(self, *args, **kwargs):
        raise NotImplementedError("vehicle tracking (KF_tracking, apis/tracking.py) is outside the device hot path; "
                                  "attach tracks with set_tracking()")

    def select_surface_wave_windows(self, x0, **kwargs):
        if not hasattr(self, "veh_states"):
            raise AttributeError("no vehicle tracks: call set_tracking() first")
        args = (self.distances_along_fiber, self.t_axis, x0, self.start_x, self.veh_states,
                self.dist_along_fiber_tracking, self.t_axis_tracking)
        self.sw_selector = SurfaceWaveSelector(self.data_for_imaging, *args, **kwargs)
        self.qs_selector = SurfaceWaveSelector(self.data, *args, **kwargs)

    def get_images(self, mute_offset=300, **imaging_kwargs):
        cls = DispersionImagesFromWindows if self.method == "surface_wave" else VirtualShotGathersFromWindows
        self.images = cls(self.sw_selector)
        self.images.get_images(mute_offset=mute_offset, **imaging_kwargs)

    def save_avg_disp_to_npz(self, *args, fdir=".", **kwargs):
        self.images.avg_image.save_to_npz(*args, fdir=fdir, **kwargs)
