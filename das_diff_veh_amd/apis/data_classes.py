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
