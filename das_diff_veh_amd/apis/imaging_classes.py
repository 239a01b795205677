"""Per-class imaging orchestration — drop-in for apis/imaging_classes.py:8-141 of the reference.

``get_images`` no longer loops over passes in Python: every window of the list goes to the device in
one batch, the class mean is produced by the fused correlate-and-stack kernel
(``dvh_vsg_stack``), and ``self.images`` (the per-pass gathers) is materialised lazily, in one
batched launch, only if a caller touches it.  ``bootstrap_disp`` (and the notebooks' ``convergence_test``) run every
resample as one device batch over gathers computed once (das_diff_veh_amd.bootstrap).
"""
from __future__ import annotations

import copy
import logging
import random

import numpy as np

from .. import engine
from .dispersion_classes import SurfaceWaveDispersion
from .virtual_shot_gather import VirtualShotGather, vsg_params


class _LazyGathers(list):
    """list of per-pass VirtualShotGather objects, computed on first access (one kernel launch)."""

    def __init__(self, windows, prm):
        super().__init__()
        self._windows, self._prm, self._done = windows, prm, False

    def _fill(self):
        if not self._done:
            self._done = True
            res, geoms = engine.gathers(self._windows, self._prm)
            super().extend(VirtualShotGather._from_arrays(w, x, g.gather_x_axis, g.gather_t_axis)
                           for w, x, g in zip(self._windows, res, geoms))

    def __len__(self):
        self._fill()
        return super().__len__()

    def __iter__(self):
        self._fill()
        return super().__iter__()

    def __getitem__(self, i):
        self._fill()
        return super().__getitem__(i)


class ImagesFromWindows:
    def __init__(self, windows, image_cls):
        self.windows = windows
        self.image_cls = image_cls

    def get_images(self, norm=False, mute_offset=300, mute=True, **imaging_kwargs):
        """Generic path (apis/imaging_classes.py:96-107): one image per window, then the mean."""
        self.images = []
        for window in self.windows:
            if mute and not window.muted_along_traj:
                window = copy.deepcopy(window)
                window.mute_along_traj(offset=mute_offset)
            self.images.append(self.image_cls(window, norm=norm, **imaging_kwargs))
        self.avg_image = sum(self.images)
        self.avg_image = self.avg_image / len(self.images)

    def save_images(self, fig_folder, file_prefix):
        """apis/imaging_classes.py:110-117: one figure per image and one of the mean, by the images' plot_image
        (plotting is outside the accelerated path: raises with a pointer before any per-pass image is formed)."""
        raise NotImplementedError(
            "plotting is outside the accelerated path (apis/imaging_classes.py:110-117 plots every image); use the "
            "reference's plot_xcorr / plot_fv_map on images[k] and avg_image"
            + ("" if getattr(self, "images", None) is not None else
               " (the per-pass images were not formed: get_images(shard_over_ranks=True) keeps only avg_image)"))


class DispersionImagesFromWindows(ImagesFromWindows):
    def __init__(self, windows, image_cls=SurfaceWaveDispersion):
        super().__init__(windows, image_cls)

    def save_images(self, fig_folder, file_prefix="veh_disp"):
        super().save_images(fig_folder, file_prefix)

    def get_images(self, norm=False, mute_offset=300, mute=True, shard_over_ranks=False, group=None,
                   **imaging_kwargs):
        """Batched flavour-B path: the trajectory mutes of all windows in one launch on a device copy
        (dvh_mute_traj), then the per-pass f-v maps and their mean on device.

        shard_over_ranks=True (torch.distributed initialised, every rank holding the same window list):
        each rank images its shard of the passes and one all-reduce of the per-class |FK| sums gives
        every rank the same ``avg_image`` (dispersion_classes.sharded_dispersion_means).  The per-pass
        images are not formed on that path: ``images`` is None and ``shard`` lists this rank's passes."""
        windows = list(self.windows)
        if shard_over_ranks:
            from .dispersion_classes import sharded_dispersion_means
            if imaging_kwargs.get("method", "naive") != "naive":
                raise ValueError("the sharded flavour-B path images method='naive' windows (the time-lapse default)")
            kw = {k: v for k, v in imaging_kwargs.items() if k != "method"}
            fv, self.shard = sharded_dispersion_means(windows, group=group, norm=norm,
                                                      mute_offset=mute_offset if mute else None, **kw)
            self.images = None
            freqs = kw.get("freqs", np.arange(0.8, 25, 0.1))
            vels = kw.get("vels", np.arange(200, 1200))
            self.avg_image = SurfaceWaveDispersion._from_fv(windows[0], freqs, vels, "naive", norm,
                                                            fv[0].to("cpu").numpy())
            return
        from .dispersion_classes import batched_surface_wave_dispersion
        self.images, self.avg_image = batched_surface_wave_dispersion(
            windows, norm=norm, mute_offset=mute_offset if mute else None, **imaging_kwargs)


class VirtualShotGathersFromWindows(ImagesFromWindows):
    def __init__(self, windows, image_cls=VirtualShotGather):
        super().__init__(windows, image_cls)

    def get_images(self, norm=False, mute_offset=300, mute=False, shard_over_ranks=False, group=None,
                   skip_failed=False, **imaging_kwargs):
        """apis/imaging_classes.py:137-138 forces norm=False, mute=False, then 96-107.

        shard_over_ranks=True (torch.distributed initialised, every rank holding the same window list):
        each rank stacks its shard of the passes with 1 / (global count) weights and one all-reduce of
        the partial stack gives every rank the same ``avg_image``; ``shard`` lists this rank's passes.
        skip_failed=True: a pass whose geometry or trajectory cannot be formed is left out of the mean
        and reported in ``failed`` {window index: reason} instead of raising for the whole list
        (engine.stacked_checked); ``images`` then holds the imaged windows' gathers.  Both flags: the
        passes every rank rejects alike are left out, the rest sharded (``shard`` in window indices)."""
        windows = list(self.windows)
        include_other_side = imaging_kwargs.pop("include_other_side", False)
        prm = vsg_params(include_other_side, norm=False, **imaging_kwargs)
        self.failed = {}
        if skip_failed and shard_over_ranks:
            # every rank holds the same list, so every rank rejects the same passes; the good ones are
            # sharded and stacked with global counts over the imaged passes
            self.failed, _ = engine.pass_failures(windows, prm)
            good = [i for i in range(len(windows)) if i not in self.failed]
            if not good:
                raise ValueError(f"no pass could be imaged: {self.failed}")
            stack, geoms, shard = engine.stacked_sharded([windows[i] for i in good], prm, group=group)
            self.shard = [good[j] for j in shard]
            self.images = _LazyGathers([windows[i] for i in good], prm)
            avg = stack[0].detach().to("cpu").numpy().astype(np.float64)
            self.avg_image = VirtualShotGather._from_arrays(windows[good[0]], avg, geoms[0].gather_x_axis,
                                                            geoms[0].gather_t_axis)
            return
        if skip_failed:
            stack, axes, self.failed = engine.stacked_checked(windows, prm)
            if stack is None:
                raise ValueError(f"no pass could be imaged: {self.failed}")
            good = [i for i in range(len(windows)) if i not in self.failed]
            self.images = _LazyGathers([windows[i] for i in good], prm)
            g0 = axes[good[0]]
            avg = stack[0].detach().to("cpu").numpy().astype(np.float64)
            self.avg_image = VirtualShotGather._from_arrays(windows[good[0]], avg, g0.gather_x_axis, g0.gather_t_axis)
            return
        if shard_over_ranks:
            stack, geoms, self.shard = engine.stacked_sharded(windows, prm, group=group)
        else:
            stack, geoms = engine.stacked(windows, prm)
        self.images = _LazyGathers(windows, prm)
        avg = stack[0].detach().to("cpu").numpy().astype(np.float64)
        self.avg_image = VirtualShotGather._from_arrays(windows[0], avg, geoms[0].gather_x_axis,
                                                        geoms[0].gather_t_axis)

    def save_images(self, fig_folder, file_prefix="veh_vshot"):
        super().save_images(fig_folder, file_prefix)


_log = logging.getLogger(__name__)


def save_disp_imgs(windows, weight, min_win, x, start_x, end_x, offset, fig_dir):
    """apis/imaging_classes.py:50-85 (imaging_diff_{speed,weight}.ipynb#cell21): the class stack of a random
    subset of min_win windows and its dispersion image.

    Same draw as the reference: ``random.sample(range(len(windows)), min_win)`` on Python's module-level
    generator (so a notebook's ``random.seed`` gives the same subset), the subset taken in window order
    (``i in sel_idx``), ``get_images(pivot=x, start_x, end_x, wlen=2, include_other_side=True)`` -- one device
    batch through the fused correlate-and-stack kernel -- and ``compute_disp_image(end_x=0, start_x=-offset)``.
    The return value is the reference's: ``images_all``, the VirtualShotGathersFromWindows of ALL windows on which
    get_images was never called (:56, :85).  The imaged subset stays reachable as ``images_all.selected`` (its
    ``avg_image.XCF_out`` / ``avg_image.disp.fv_map``) and the draw as ``images_all.sel_idx``, attributes the
    reference does not have.  Not done (plotting is outside the accelerated path): the figures the reference
    writes under ``fig_dir/x/`` (plot_image of the stack, plot_fv_map with and without normalisation) and the
    CLAHE enhancement (fv_map_enhance, cv2), whose result the reference only passes to a commented-out plot."""
    image_from_window_cls = VirtualShotGathersFromWindows
    sel_idx = random.sample(range(len(windows)), min_win)
    images_all = image_from_window_cls(windows)
    chosen = set(sel_idx)
    _images = image_from_window_cls([e for i, e in enumerate(windows) if i in chosen])
    _images.get_images(pivot=x, start_x=start_x, end_x=end_x, wlen=2, include_other_side=True)
    _log.info("save_disp_imgs: figures sg_%s_cars.pdf / disp_%s_cars_no_norm.pdf / disp_%s_cars_no_enhance.pdf under "
              "%s/%s/ are not written (plotting is outside the accelerated path; plot images.selected.avg_image with "
              "the reference's plot_xcorr / plot_fv_map)", weight, weight, weight, fig_dir, x)
    _images.avg_image.compute_disp_image(end_x=0, start_x=-offset)
    images_all.selected, images_all.sel_idx = _images, sel_idx
    return images_all


def bootstrap_disp(surf_wins, bt_size, bt_times, sigma, pivot, start_x, end_x, ref_freq_idx, freq_lb, freq_up,
                   ref_vel):
    """apis/imaging_classes.py:8-48: bt_times resamples of random.sample(range(1, n), bt_size)
    windows -> class-stack VSG -> compute_disp_image(end_x=0, start_x=-150) -> one ridge per mode.
    Same draws (Python ``random``), same return value: (ridge_vel[mode][resample], freqs).  All
    resamples run as one batch on the device (das_diff_veh_amd.bootstrap)."""
    from .. import bootstrap as bt
    cache = bt.GatherCache(surf_wins, pivot, start_x, end_x)
    sels = bt.draw(len(surf_wins), bt_size, bt_times)
    per_mode = bt.bootstrap_ridges(cache, sels, sigma, ref_freq_idx, freq_lb, freq_up, ref_vel)
    return [list(r) for r in per_mode], bt.FREQS.copy()


def convergence_test(max_sample_num, windows, bt_times, sigma, x0, start_x, end_x, ref_freq_idx, freq_lb, freq_ub,
                     vel_ref):
    """imaging_diff_speed.ipynb#cell30: for bt_size = 1..max_sample_num, the summed per-frequency
    std of the bootstrap ridges -> [n_modes, max_sample_num].  The gathers are computed once for all
    60 x bt_times resamples (the notebook recomputes them per resample); draws as the notebook's; all
    resamples imaged in one batch (das_diff_veh_amd.bootstrap.convergence)."""
    from .. import bootstrap as bt
    cache = bt.GatherCache(windows, x0, start_x, end_x)
    return bt.convergence(cache, max_sample_num, bt_times, sigma, ref_freq_idx, freq_lb, freq_ub, vel_ref)
