"""save_disp_imgs (apis/imaging_classes.py:50-85, imaging_diff_{speed,weight}.ipynb#cell21) in the drop-in: the
same random.sample draw as the reference, the subset's class stack and f-v image against the reference's golden
gathers and the oracle's map_fv (tol 1e-4, picks under SURVEY §8d's tie rule), and the reference's return value
(the un-imaged VirtualShotGathersFromWindows of all windows)."""
import random

import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.mark.parametrize("seed,min_win,offset", [(11, 3, 200), (2024, 4, 150)])
def test_save_disp_imgs_subset_stack_and_image(device, tmp_path, seed, min_win, offset):
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows, save_disp_imgs
    from oracle import disp as odisp
    g = gio.load("vsg_w500")
    n = gio.n_pass(g)
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(n)]
    # the reference's draw on Python's module-level generator, and what the generator gives next
    random.seed(seed)
    ref_idx = random.sample(range(n), min_win)
    nxt = random.random()
    random.seed(seed)
    images_all = save_disp_imgs(wins, "fast", min_win, 700, 500, 900, offset, str(tmp_path))
    assert random.random() == nxt  # the drop-in consumed exactly the reference's draws
    assert images_all.sel_idx == ref_idx
    # the reference returns images_all, built from every window, on which get_images was never called
    assert isinstance(images_all, VirtualShotGathersFromWindows) and images_all.windows == wins
    assert not hasattr(images_all, "avg_image") and not hasattr(images_all, "images")
    sub = images_all.selected
    assert [id(w) for w in sub.windows] == [id(wins[i]) for i in sorted(ref_idx)]  # window order, not draw order
    ref_stack = np.mean([g["xcf"][i] for i in sorted(ref_idx)], axis=0)
    assert gio.gather_rel_err(sub.avg_image.XCF_out, ref_stack) < TOL
    avg = sub.avg_image
    fv_ref = odisp.compute_disp_image(ref_stack, avg.x_axis, avg.t_axis, start_x=-offset, end_x=0)
    fv = avg.disp.fv_map
    assert fv.shape == fv_ref.shape == (1000, 242)
    assert np.abs(fv - fv_ref).max() / np.abs(fv_ref).max() < TOL
    assert np.all(odisp.pick_ok(fv_ref, fv.argmax(axis=0)))
    assert not any(tmp_path.iterdir())  # no figures are written (plotting is outside the accelerated path)


def test_save_images_points_at_plotting(device, tmp_path):
    """ImagesFromWindows.save_images (apis/imaging_classes.py:110-117) exists on the drop-in classes and raises with a
    pointer to the reference's plotting, without materialising the per-pass gathers first."""
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows
    g = gio.load("vsg_w500")
    images = VirtualShotGathersFromWindows([SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(2)])
    images.get_images(include_other_side=True, pivot=700, start_x=500, end_x=900, wlen=2)
    with pytest.raises(NotImplementedError, match="plot"):
        images.save_images(str(tmp_path))
    assert not images.images._done  # the lazily computed per-pass gathers were not formed
