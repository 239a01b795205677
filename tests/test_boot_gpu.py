"""GPU parity of the bootstrap path: ridge walk, resample stacks, end-to-end
bootstrap_disp / convergence_test against the reference's goldens (tests/golden/ridge.npz) and the
oracle (oracle/ridge.py)."""
import random

import numpy as np
import pytest
import scipy.interpolate

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
KW = dict(pivot=700, start_x=500, end_x=900)


def _mode1(g):
    return scipy.interpolate.interp1d(g["refvel_f"], g["refvel_v"])


def test_ridge_kernel_matches_reference_goldens(device):
    """dvh_ridge on the reference's own f-v map gives the reference's ridges (walk, reference curve,
    vel_max modes of extract_ridge_ref_idx)."""
    import torch

    from das_diff_veh_amd.bootstrap import ridges
    g = gio.load("ridge")
    fq, vels = g["freqs"], g["vels"]
    fv = torch.as_tensor(g["fv_map"].astype(np.float32), device=device)[None]
    w = ridges(fv, fq, vels, 2.5, 14, ref_freq_idx=80 - int(np.sum(fq < 2.5)), sigma=25, vel_max=800)[0]
    np.testing.assert_allclose(w, g["walk"], rtol=0, atol=1e-9)
    r = ridges(fv, fq, vels, 10, 15, ref_freq_idx=130 - int(np.sum(fq < 10)), sigma=50, vel_max=800,
               ref_vel=_mode1(g))[0]
    np.testing.assert_allclose(r, g["refvel"], rtol=0, atol=1e-9)
    v = ridges(fv, fq, vels, 2.5, 14, sigma=25, vel_max=800)[0]
    np.testing.assert_array_equal(v, g["velmax"])


def test_extract_ridge_mirror(device):
    from das_diff_veh_amd.modules.utils import extract_ridge_ref_idx
    g = gio.load("ridge")
    fq, vels, fv = g["freqs"], g["vels"], g["fv_map"]
    m = (fq >= 2.5) & (fq < 14)
    w = extract_ridge_ref_idx(fq[m], vels, fv[:, m], ref_freq_idx=80 - int(np.sum(fq < 2.5)), sigma=25, vel_max=800)
    np.testing.assert_allclose(w, g["walk"], rtol=0, atol=1e-9)
    with pytest.raises(ValueError):  # savgol window longer than the band, as scipy raises
        extract_ridge_ref_idx(fq[:10], vels, fv[:, :10], ref_freq_idx=3)


def _windows():
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    g = gio.load("vsg_w500")
    return [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(gio.n_pass(g))], g


def test_resample_stacks_and_images(device):
    """Resample stacks = mean of the drawn passes' gathers; their f-v images = map_fv of the oracle."""
    from das_diff_veh_amd import bootstrap as bt
    from oracle import disp as odisp
    from oracle import vsg as ovsg
    wins, g = _windows()
    cache = bt.GatherCache(wins, **KW)
    sels = np.array([[1, 3, 4], [2, 2, 1], [4, 1, 2]], dtype=np.int32)
    stacks = cache.resample_stacks(sels).double().cpu().numpy()
    fv = cache.resample_images(sels).cpu().numpy()
    s, e, _ = cache.disp_plan()
    for b, sel in enumerate(sels):
        ref = ovsg.stack([g["xcf"][i] for i in sel])
        assert gio.gather_rel_err(stacks[b], ref[s:e + 1]) < 1e-4
        rfv = odisp.compute_disp_image(ref, g["gather_x_axis"], g["gather_t_axis"], start_x=-150, end_x=0)
        assert np.abs(fv[b] - rfv).max() <= 1e-4 * np.abs(rfv).max()


def test_bootstrap_disp_matches_reference(device):
    """Same draws as the reference (random.seed); ridges identical to the oracle's on our own images
    (the walk's logic), and to the reference's ridges up to the f-v parity (1e-4)."""
    from das_diff_veh_amd import bootstrap as bt
    from das_diff_veh_amd.apis.imaging_classes import bootstrap_disp
    from oracle import ridge as orid
    wins, _ = _windows()
    g = gio.load("ridge")
    mode1 = _mode1(g)
    random.seed(11)
    rv, fq = bootstrap_disp(wins, 3, 4, [25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    np.testing.assert_array_equal(fq, g["boot_freqs"])
    random.seed(11)
    sels = bt.draw(len(wins), 3, 4)
    np.testing.assert_array_equal(sels, g["boot_sel"])
    # the ridge walk on our images equals the oracle's walk on the same images
    cache = bt.GatherCache(wins, **KW)
    fv = cache.resample_images(sels).cpu().numpy()
    for b in range(4):
        for m, (lb, ub, ri, sg, vr) in enumerate(((2.5, 14, 80, 25, None), (10, 15, 130, 50, mode1))):
            band = (fq >= lb) & (fq < ub)
            o = orid.extract_ridge_ref_idx(fq[band], bt.VELS, fv[b][:, band], ref_freq_idx=ri - int(np.sum(fq < lb)),
                                           sigma=sg, vel_max=800, ref_vel=vr)
            np.testing.assert_allclose(rv[m][b], o, rtol=0, atol=1e-9)
    # and the reference's ridges (its f-v maps differ from ours by <= 1e-4 relative; the picks agree)
    for m, key in enumerate(("boot_mode0", "boot_mode1")):
        d = np.abs(np.stack(rv[m]) - g[key])
        assert d.max() <= 2.0 and d.mean() <= 0.1, (m, d.max(), d.mean())


def test_convergence_test_small(device):
    from das_diff_veh_amd.apis.imaging_classes import convergence_test
    from oracle import ridge as orid
    wins, g5 = _windows()
    g = gio.load("ridge")
    mode1 = _mode1(g)
    args = ([25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    random.seed(5)
    got = convergence_test(3, wins, 4, *args)
    random.seed(5)
    ow = [gio.oracle_window(g5, i) for i in range(len(wins))]
    ref = np.empty_like(got)
    for k in range(1, 4):
        rv, _ = orid.bootstrap_disp(ow, k, 4, *args)
        for m in range(2):
            ref[m, k - 1] = np.sum(np.std(rv[m], axis=0))
    np.testing.assert_allclose(got, ref, rtol=0.05, atol=2.0)
