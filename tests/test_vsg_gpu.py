"""GPU parity of the VSG kernels against the reference's golden vectors (tol 1e-4, fp32 vs float64)."""
import ast

import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _windows(g, prefix="", n=None):
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    n = gio.n_pass(g, prefix) if n is None else n
    return [SurfaceWaveWindow(**gio.pass_arrays(g, i, prefix)) for i in range(n)]


KW = dict(pivot=700, start_x=500, end_x=900, wlen=2)


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
def test_per_pass_gathers(device, fixture):
    from das_diff_veh_amd import engine
    from das_diff_veh_amd.plan import VsgParams
    g = gio.load(fixture)
    wins = _windows(g)
    res, geoms = engine.gathers(wins, VsgParams(include_other_side=True, norm=False, **KW), device=device)
    for i, x in enumerate(res):
        err = gio.gather_rel_err(x, g["xcf"][i])
        assert err < TOL, (fixture, i, err)
    if "gather_t_axis" in g:
        assert np.array_equal(geoms[0].gather_t_axis, g["gather_t_axis"])


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
def test_class_stack(device, fixture):
    from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows
    g = gio.load(fixture)
    images = VirtualShotGathersFromWindows(_windows(g))
    images.get_images(include_other_side=True, **KW)
    err = gio.gather_rel_err(images.avg_image.XCF_out, g["stack"])
    assert err < TOL, err
    # the lazily materialised per-pass images agree too
    for i, im in enumerate(images.images):
        assert gio.gather_rel_err(im.XCF_out, g["xcf"][i]) < TOL


@pytest.mark.parametrize("name,kw", [
    ("xcf_norm_2s", dict(include_other_side=True)),
    ("xcf_norm_1s", dict(include_other_side=False)),
    ("xcf_nonorm_1s", dict(include_other_side=False, norm=False)),
    ("xcf_raw_2s", dict(include_other_side=True, norm=False, norm_amp=False)),
])
def test_direct_constructor_variants(device, name, kw):
    from das_diff_veh_amd.apis.virtual_shot_gather import VirtualShotGather
    g = gio.load("vsg_w500")
    win = _windows(g, n=1)[0]
    vsg = VirtualShotGather(win, **kw, **KW)
    assert gio.gather_rel_err(vsg.XCF_out, g[name][0]) < TOL


@pytest.mark.parametrize("case", ["early", "late", "slow", "p680", "narrow", "wlen1"])
def test_edge_cases(device, case):
    from das_diff_veh_amd.apis.virtual_shot_gather import VirtualShotGather
    g = gio.load("vsg_edge")
    win = _windows(g, prefix=case + "_", n=1)[0]
    kw = ast.literal_eval(str(g[case + "_kw"]))
    vsg = VirtualShotGather(win, include_other_side=True, norm=False, **kw)
    assert gio.gather_rel_err(vsg.XCF_out, g[case + "_xcf"]) < TOL
    assert np.array_equal(vsg.x_axis, g[case + "_gx"])
    assert np.array_equal(vsg.t_axis, g[case + "_gt"])
