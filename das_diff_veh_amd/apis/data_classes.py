"""SurfaceWaveWindow — the unit of work of the hot path (mirror of apis/data_classes.py:12-123).

Same constructor, attributes and mutating methods as the reference.  ``data`` may be a NumPy array
(as in the pickled notebook windows) or a device tensor; the mutes run as HIP kernels on a device
copy and write the result back into the same container type, in place, like the reference.
"""
from __future__ import annotations

import numpy as np

from ..plan import interp1d_extrap


class SurfaceWaveWindow:
    def __init__(self, data, x_axis, t_axis, veh_state, start_x_tracking, distance_along_fiber_tracking,
                 t_axis_tracking):
        self.data = data
        self.x_axis = x_axis
        self.t_axis = t_axis
        self.veh_state = veh_state
        self.start_x_tracking = start_x_tracking
        self.distance_along_fiber_tracking = distance_along_fiber_tracking
        self.t_axis_tracking = t_axis_tracking
        self.muted_along_traj = False
        self.muted_along_time = False
        self._preprocess_veh_state()

    def _preprocess_veh_state(self):
        """apis/data_classes.py:34-39: tracking indices -> (distance [m], time [s]) samples."""
        vs = np.asarray(self.veh_state, dtype=np.float64)
        ok = ~np.isnan(vs)
        tmp = vs[ok].astype(int)
        i0 = np.abs(self.start_x_tracking - np.asarray(self.distance_along_fiber_tracking)).argmin()
        self.veh_state_x = np.asarray(self.distance_along_fiber_tracking)[np.where(ok)[0] + i0]
        self.veh_state_t = np.asarray(self.t_axis_tracking)[tmp]

    def trajectory(self):
        """f(x) -> t, the interp1d(..., fill_value='extrapolate') the VSG path builds."""
        return interp1d_extrap(self.veh_state_x, self.veh_state_t)

    def mute_along_traj(self, offset=200, alpha=0.3, delta_x=20):
        """apis/data_classes.py:49-72, on device (HIP kernel dvh_mute_traj)."""
        from ..preprocess import mute_along_traj
        mute_along_traj(self, offset=offset, alpha=alpha, delta_x=delta_x)
        self.muted_along_traj = True

    def mute_along_time(self, alpha=0.3):
        """apis/data_classes.py:100-104, on device (HIP kernel dvh_mute_time)."""
        from ..preprocess import mute_along_time
        mute_along_time(self, alpha=alpha)
        self.muted_along_time = True

    def plot_on_data(self, ax, c="r"):
        import matplotlib.patches as patches
        length_sw = self.x_axis[-1] - self.x_axis[0]
        wlen_sw = self.t_axis[-1] - self.t_axis[0]
        ax.add_patch(patches.Rectangle((self.x_axis[0], self.t_axis[0]), length_sw, wlen_sw, linewidth=1,
                                       edgecolor=c, facecolor="none"))


class SurfaceWaveSelector:
    """apis/data_classes.py:126-255: one SurfaceWaveWindow per isolated pass at x0.

    Same constructor, attributes and container protocol as the reference.  The index bookkeeping is
    ``select.pass_table`` (host, O(n_passes)); the window copies are cut on the device in one launch
    per window shape (dvh_cut_windows).  A host record gives host windows (float64 copies, as the
    reference's deepcopy); a device record gives device windows.  ``batch`` holds the device batch
    [n_win, n_ch, n_t] when all windows share one shape (the input of the imaging kernels)."""

    def __init__(self, data_for_surface_wave, distances_along_fiber, t_axis, x0, start_x_tracking, veh_states,
                 distance_along_fiber_tracking, t_axis_tracking, wlen_sw=8, length_sw=300, spatial_ratio=0.75,
                 temporal_spacing=None):
        self.data_for_surface_wave = data_for_surface_wave
        self.distances_along_fiber = distances_along_fiber
        self.t_axis = t_axis
        self.dt = self.t_axis[1] - self.t_axis[0]
        self.x0 = x0
        self.start_x_tracking = start_x_tracking
        self.veh_states = veh_states
        self.distance_along_fiber_tracking = distance_along_fiber_tracking
        self.t_axis_tracking = t_axis_tracking
        self.wlen_sw = wlen_sw
        self.length_sw = length_sw
        self.spatial_ratio = spatial_ratio
        self.temporal_spacing = temporal_spacing if temporal_spacing else self.wlen_sw
        self.locate_windows()

    def locate_windows(self):
        import torch

        from ..select import cut_windows, pass_table, record_on_device
        ks, xr, t0, t1 = pass_table(self.t_axis, self.distances_along_fiber, self.x0, self.start_x_tracking,
                                    self.veh_states, self.t_axis_tracking, self.dt, wlen_sw=self.wlen_sw,
                                    length_sw=self.length_sw, spatial_ratio=self.spatial_ratio,
                                    temporal_spacing=self.temporal_spacing)
        self.pass_indices = ks
        self.batch = None
        if ks.size == 0:
            self.windows = []
            return
        d = self.data_for_surface_wave
        on_device = isinstance(d, torch.Tensor) and d.is_cuda
        batches, where = cut_windows(record_on_device(d), xr, t0, t1)
        if len(batches) == 1:
            self.batch = next(iter(batches.values()))
        if not on_device:  # host windows: one download per batch, numpy views into it
            batches = {n: b.cpu().numpy() for n, b in batches.items()}
        views = [batches[n][j] for n, j in where]
        xa = np.asarray(self.distances_along_fiber)[xr[0]:xr[1]]
        ta = np.asarray(self.t_axis)
        vs = self.veh_states
        self.windows = [SurfaceWaveWindow(data=v, t_axis=ta[a:b], x_axis=xa, veh_state=vs[k],
                                          start_x_tracking=self.start_x_tracking,
                                          distance_along_fiber_tracking=self.distance_along_fiber_tracking,
                                          t_axis_tracking=self.t_axis_tracking)
                        for v, k, a, b in zip(views, ks, t0, t1)]

    def __len__(self):
        return len(self.windows)

    def __getitem__(self, item):
        return self.windows[item]

    def __setitem__(self, key, value):
        self.windows[key] = value

    def __contains__(self, item):
        return 0 <= item < len(self.windows)
