"""ImagingWorkflowOneDirectory — the daily loop of apis/imaging_workflow.py:21-80 over the device classes.

The reference reads a directory of records with ImagingIO (modules/imaging_IO.py) and tracks each record's vehicles
with KF_tracking; both are outside the device hot path.  Here the records are any iterable of
``(data, x_axis, t_axis)`` -- what ImagingIO yields -- and the tracks come from ``tracks(k, imagingObj)``, a callable
returning record k's tracking results ``(veh_states, dist_along_fiber_tracking, t_axis_tracking)`` (what
track_cars / _preprocess_for_tracking leave on the object), or from a list of such tuples; ``imaging``'s start_x /
end_x are the tracking span, as the reference passes them to track_cars.  The loop body is the reference's:
TimeLapseImaging -> select_surface_wave_windows -> get_images -> ``avg_image += images.avg_image`` (a sum of the
per-record means, starting from 0), snapshots every ``n_min_save`` minutes, then ``save_avg_disp_to_npz``.
"""
from __future__ import annotations

from .timeLapseImaging import TimeLapseImaging


class ImagingWorkflowOneDirectory:
    def __init__(self, records, tracks, method="surface_wave", time_interval=60.0, directory=None):
        """records: iterable of (data, x_axis, t_axis); tracks: callable (k, imagingObj) -> (veh_states,
        dist_along_fiber_tracking, t_axis_tracking), or a sequence of them; time_interval: seconds per record
        (ImagingIO.get_time_interval)."""
        self.records = records
        self.tracks = tracks
        self.method = method
        self.time_interval = time_interval
        self.directory = directory

    def _tracks_of(self, k, obj):
        return self.tracks(k, obj) if callable(self.tracks) else self.tracks[k]

    def imaging(self, start_x, end_x, x0, wlen_sw=8, length_sw=300, spatial_ratio=0.75, n_min_save=30,
                temporal_spacing=None, num_to_stop=None, verbal=True, surface_wave_preprecessing_dict=None,
                imaging_kwargs=None):
        """apis/imaging_workflow.py:33-80.  start_x / end_x: the tracking span (track_cars(start_x, end_x): start_x is
        the selector's start_x_tracking); imaging_kwargs go to get_images (the reference requires them: its default None fails
        at ``**imaging_kwargs``)."""
        if imaging_kwargs is None:
            raise TypeError("imaging_kwargs is required (the reference's get_images(**None) raises)")
        avg_image = 0
        num_veh = 0
        self.avg_images_to_save = []
        n_win_save = int(n_min_save * 60 / self.time_interval)
        for k, (data, x_axis, t_axis) in enumerate(self.records):
            if num_to_stop and k >= num_to_stop:
                break
            if verbal:
                print(f"working on window {k}, method={self.method}")
            obj = TimeLapseImaging(data, x_axis, t_axis, method=self.method,
                                   surface_wave_preprecessing_dict=surface_wave_preprecessing_dict)
            veh_states, dist_trk, t_trk = self._tracks_of(k, obj)
            obj.set_tracking(veh_states, start_x, dist_trk, t_trk, end_x=end_x)
            obj.select_surface_wave_windows(x0=x0, wlen_sw=wlen_sw, length_sw=length_sw, spatial_ratio=spatial_ratio,
                                            temporal_spacing=temporal_spacing)
            n_cur = len(obj.sw_selector)
            if n_cur == 0:
                continue
            num_veh += n_cur
            obj.get_images(**imaging_kwargs)
            avg_image += obj.images.avg_image
            if k == 0 or (k + 1) % n_win_save == 0:
                self.avg_images_to_save.append({"avg_image": avg_image, "time": k * n_min_save, "num_veh": num_veh})
        self.avg_image = avg_image
        self.num_veh = num_veh

    def save_avg_disp_to_npz(self, *args, fdir=None, **kwargs):
        """apis/imaging_workflow.py:97-98."""
        self.avg_image.save_to_npz(*args, fdir=fdir, **kwargs)

    def plot_avg_images(self, *args, **kwargs):
        raise NotImplementedError("plotting is outside the accelerated path; use the reference's plot_image on "
                                  "avg_image")

    plot_intermediate_images = plot_avg_images
