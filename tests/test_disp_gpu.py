"""GPU parity of the dispersion kernels (map_fv) against the reference's golden f-v maps.

Contract (north_star / SURVEY §8(d)): f-v values within rel-err 1e-4 of the reference (max abs error
over the map / max |map|), and the dispersion-curve pick identical: for every frequency column the
build's argmax over velocity must hit the reference's maximum value (ties in the float32 reference
are allowed; strict index identity is asserted separately where the reference has no near-tie).
"""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _fv_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max())


def _picks_ok(got, ref):
    from oracle.disp import pick_ok
    return pick_ok(ref, np.argmax(got, axis=0))


def _check(got, ref):
    assert got.shape == ref.shape
    assert _fv_err(got, ref) < TOL
    ok = _picks_ok(got, ref)
    assert ok.all(), f"{(~ok).sum()} of {ok.size} picks miss the reference maximum"


@pytest.mark.parametrize("fixture,key,norm", [("vsg_w500", "fv_map", False), ("vsg_w500", "fv_map_l1", True),
                                              ("vsg_w499", "fv_map", False)])
def test_stack_dispersion(device, fixture, key, norm):
    from das_diff_veh_amd.apis.virtual_shot_gather import VirtualShotGather
    g = gio.load(fixture)
    x = gio.load("vsg_w500")
    gt = g["gather_t_axis"]
    vsg = VirtualShotGather._from_arrays(None, g["stack"], x["gather_x_axis"], gt)
    vsg.compute_disp_image(end_x=0, start_x=-200, norm=norm)
    _check(vsg.disp.fv_map, g[key])


def _disp_windows():
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    g = gio.load("disp")
    return g, [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(gio.n_pass(g))]


def test_naive_per_pass_and_stack(device):
    from das_diff_veh_amd.apis.dispersion_classes import SurfaceWaveDispersion
    g, wins = _disp_windows()
    ims = [SurfaceWaveDispersion(w, freqs=g["freqs"], vels=g["vels"], method="naive", norm=False, start_x=500,
                                 end_x=800) for w in wins]
    for i, im in enumerate(ims):
        _check(im.disp.fv_map, g["naive_fv"][i])
    avg = sum(ims) / len(ims)
    _check(avg.disp.fv_map, g["naive_stack"])
    l1 = SurfaceWaveDispersion(wins[0], freqs=g["freqs"], vels=g["vels"], method="naive", norm=True, start_x=500,
                               end_x=800)
    _check(l1.disp.fv_map, g["naive_l1_fv"])


def test_smart_disp(device):
    from das_diff_veh_amd.apis.dispersion_classes import SurfaceWaveDispersion
    g, wins = _disp_windows()
    im = SurfaceWaveDispersion(wins[1], freqs=g["freqs"], vels=g["vels"], method="smart", norm=False)
    _check(im.disp.fv_map, g["smart_fv"])


def test_dispersion_images_from_windows(device):
    from das_diff_veh_amd.apis.imaging_classes import DispersionImagesFromWindows
    g, wins = _disp_windows()
    imgs = DispersionImagesFromWindows(wins)
    imgs.get_images(mute_offset=300, freqs=g["freqs"], vels=g["vels"], method="naive", start_x=500, end_x=800)
    _check(imgs.avg_image.disp.fv_map, g["muted_stack"])
    # the caller's windows are not muted (deep copies), like the reference
    assert not any(w.muted_along_traj for w in wins)


def test_mutes(device):
    g, wins = _disp_windows()
    import copy
    w = copy.deepcopy(wins[2])
    w.data = w.data.astype(np.float64)
    w.mute_along_traj(offset=300)
    assert np.abs(w.data.astype(np.float32) - g["mute_traj_300"]).max() <= 1e-7
    w = copy.deepcopy(wins[2])
    w.mute_along_time(alpha=0.3)
    assert np.abs(w.data - g["mute_time_03"]).max() <= 2e-7


@pytest.mark.parametrize("key,flo,fhi", [("out_1p2_30", 1.2, 30), ("out_0p08_1", 0.08, 1)])
def test_bandpass(device, key, flo, fhi):
    from das_diff_veh_amd.modules.utils import bandpass_data
    g = gio.load("bandpass")
    x = g["q"].astype(np.float64) * 2.0 ** -12
    bandpass_data(x, float(g["dt"]), flo, fhi)
    ref = g[key]
    assert np.abs(x - ref).max() / np.abs(ref).max() < 1e-10
    # float32 device data (the hot-path dtype) stays within fp32 rounding of the float64 result
    x32 = (g["q"].astype(np.float32) * np.float32(2.0 ** -12))
    bandpass_data(x32, float(g["dt"]), flo, fhi)
    assert np.abs(x32 - ref).max() / np.abs(ref).max() < 1e-6
