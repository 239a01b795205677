"""The oracle (CPU restatement) against the reference's golden vectors: this is what pins it."""
import ast

import numpy as np
import pytest

from tests import golden_io as gio

KW = dict(pivot=700, start_x=500, end_x=900, wlen=2)


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
def test_vsg_per_pass_and_stack(fixture):
    from oracle import vsg
    g = gio.load(fixture)
    xs = []
    for i in range(gio.n_pass(g)):
        x, gx, gt = vsg.virtual_shot_gather(gio.oracle_window(g, i), include_other_side=True, norm=False, **KW)
        assert np.abs(x - g["xcf"][i]).max() < 1e-12
        xs.append(x)
    assert np.abs(vsg.stack(xs) - g["stack"]).max() < 1e-12
    assert np.array_equal(gt, g["gather_t_axis"])


@pytest.mark.parametrize("name,kw", [
    ("xcf_norm_2s", dict(include_other_side=True)),
    ("xcf_norm_1s", dict(include_other_side=False)),
    ("xcf_nonorm_1s", dict(include_other_side=False, norm=False)),
    ("xcf_raw_2s", dict(include_other_side=True, norm=False, norm_amp=False)),
])
def test_vsg_variants(name, kw):
    from oracle import vsg
    g = gio.load("vsg_w500")
    x, _, _ = vsg.virtual_shot_gather(gio.oracle_window(g, 0), **kw, **KW)
    ref = g[name][0]
    assert np.array_equal(np.isnan(x), np.isnan(ref))
    m = np.isfinite(ref)
    assert np.abs(x[m] - ref[m]).max() <= 1e-12 * max(1.0, np.abs(ref[m]).max())


@pytest.mark.parametrize("case", ["early", "late", "slow", "p680", "narrow", "wlen1"])
def test_vsg_edges(case):
    from oracle import vsg
    g = gio.load("vsg_edge")
    kw = ast.literal_eval(str(g[case + "_kw"]))
    x, gx, gt = vsg.virtual_shot_gather(gio.oracle_window(g, 0, case + "_"), include_other_side=True, norm=False,
                                        **kw)
    ref = g[case + "_xcf"]
    assert x.shape == ref.shape
    assert np.array_equal(np.isnan(x), np.isnan(ref)) and np.array_equal(np.isinf(x), np.isinf(ref))
    m = np.isfinite(ref)
    if m.any():
        assert np.abs(x[m] - ref[m]).max() < 1e-12
    assert np.array_equal(gx, g[case + "_gx"]) and np.array_equal(gt, g[case + "_gt"])


def test_vsg_dt_exact_raises_like_reference():
    from das_diff_veh_amd.synth import synth_pass
    from oracle import vsg
    g = gio.load("vsg_edge")
    assert bool(g["dt004_raises"])
    p = synth_pass(306, t0=0.0)
    w = vsg.window_from_arrays(p["q"], p["x_axis"], p["t_axis"], p["veh_state"], p["start_x_tracking"],
                               p["distance_along_fiber_tracking"], p["t_axis_tracking"])
    with pytest.raises(ValueError):
        vsg.virtual_shot_gather(w, include_other_side=True, norm=False, **KW)


def test_disp_stack_images():
    from oracle import disp
    g = gio.load("vsg_w500")
    fv = disp.compute_disp_image(g["stack"], g["gather_x_axis"], g["gather_t_axis"], start_x=-200, end_x=0)
    assert np.array_equal(fv, g["fv_map"])
    fv = disp.compute_disp_image(g["stack"], g["gather_x_axis"], g["gather_t_axis"], start_x=-200, end_x=0, norm=True)
    assert np.array_equal(fv, g["fv_map_l1"])


def test_disp_per_pass_and_mutes():
    from oracle import disp, preprocess, vsg
    g = gio.load("disp")
    fr, vl = g["freqs"], g["vels"]
    wins = [gio.oracle_window(g, i) for i in range(gio.n_pass(g))]
    fvs = [disp.naive_disp(w["data"], w["x_axis"], w["t_axis"], fr, vl, 500, 800, norm=False) for w in wins]
    for i, fv in enumerate(fvs):
        assert np.array_equal(fv, g["naive_fv"][i])
    assert np.abs(sum(fvs) / 3 - g["naive_stack"]).max() == 0
    w = wins[2]
    m = preprocess.mute_along_traj(w["data"], w["x_axis"], w["t_axis"], w["veh_state_x"], w["veh_state_t"], 300)
    assert np.array_equal(m.astype(np.float32), g["mute_traj_300"])
    assert np.array_equal(preprocess.mute_along_time(w["data"], 0.3).astype(np.float32), g["mute_time_03"])
    _ = vsg


def test_bandpass():
    from oracle import preprocess
    g = gio.load("bandpass")
    x = g["q"][:2].astype(np.float64) * 2.0 ** -12
    y = preprocess.bandpass_data(x, float(g["dt"]), 1.2, 30)
    assert np.abs(y - g["out_1p2_30"][:2]).max() < 1e-12


def test_ref_loop_baseline_matches_reference():
    """The CPU baseline bench.py times computes the reference's results."""
    from oracle import ref_loop
    g = gio.load("vsg_w500")
    gs = []
    for i in range(2):
        w = gio.oracle_window(g, i)
        x, gx, gt = ref_loop.gather(w["data"], w["x_axis"], w["t_axis"], w["veh_state_x"], w["veh_state_t"], 700, 500,
                                    900)
        assert np.abs(x - g["xcf"][i]).max() < 1e-12
        gs.append(x)
    fv = ref_loop.disp_image(g["stack"], g["gather_x_axis"], g["gather_t_axis"])
    assert np.abs(fv - g["fv_map"]).max() <= 1e-6 * np.abs(g["fv_map"]).max()


def test_oracle_ridge_and_bootstrap_match_reference():
    """oracle/ridge.py against the reference's extract_ridge_ref_idx and bootstrap_disp
    (tests/golden/ridge.npz, random.seed(11))."""
    import random

    import scipy.interpolate

    from oracle import ridge as orid
    g = gio.load("ridge")
    fq, vels, fv = g["freqs"], g["vels"], g["fv_map"]
    m0, m1 = (fq >= 2.5) & (fq < 14), (fq >= 10) & (fq < 15)
    mode1 = scipy.interpolate.interp1d(g["refvel_f"], g["refvel_v"])
    assert np.array_equal(orid.extract_ridge_ref_idx(fq[m0], vels, fv[:, m0], ref_freq_idx=80 - int(np.sum(fq < 2.5)),
                                                     sigma=25, vel_max=800), g["walk"])
    assert np.array_equal(orid.extract_ridge_ref_idx(fq[m1], vels, fv[:, m1], ref_freq_idx=130 - int(np.sum(fq < 10)),
                                                     sigma=50, vel_max=800, ref_vel=mode1), g["refvel"])
    assert np.array_equal(orid.extract_ridge_ref_idx(fq[m0], vels, fv[:, m0], sigma=25, vel_max=800), g["velmax"])
    assert np.array_equal(orid.extract_ridge_ref_idx(fq[m0], vels, fv[:, m0], ref_freq_idx=-7, sigma=25, vel_max=800),
                          g["walk_neg7"])
    v5 = gio.load("vsg_w500")
    wins = [gio.oracle_window(v5, i) for i in range(5)]
    random.seed(11)
    rv, f = orid.bootstrap_disp(wins, 3, 4, [25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    assert np.abs(np.stack(rv[0]) - g["boot_mode0"]).max() < 1e-9
    assert np.abs(np.stack(rv[1]) - g["boot_mode1"]).max() < 1e-9
    # the reference's per-resample f-v maps (boot_fv) give its bootstrap ridges through the oracle walk
    for b in range(4):
        for m, (lb, ub, ri, sg, vr, key) in enumerate(((2.5, 14, 80, 25, None, "boot_mode0"),
                                                       (10, 15, 130, 50, mode1, "boot_mode1"))):
            band = (f >= lb) & (f < ub)
            r = orid.extract_ridge_ref_idx(f[band], vels, g["boot_fv"][b][:, band], ref_freq_idx=ri - int(np.sum(f < lb)),
                                           sigma=sg, vel_max=800, ref_vel=vr)
            assert np.abs(r - g[key][b]).max() < 1e-9, (b, m)


@pytest.mark.parametrize("case", ["stack", "odd", "pow2"])
def test_oracle_fk_matches_reference(case):
    """oracle/disp.fk against the reference's fk (modules/utils.py:236-248): magnitudes and both axes."""
    from oracle import disp as odisp
    g = gio.load("fk")
    res, ff, kk = odisp.fk(g[case + "_data"], float(g[case + "_dx"]), float(g[case + "_dt"]))
    ref = g[case + "_fk"].astype(np.float64)
    assert res.shape == ref.shape
    assert np.abs(res - ref).max() <= 1e-6 * np.abs(ref).max()
    assert np.array_equal(ff, g[case + "_f"]) and np.array_equal(kk, g[case + "_k"])


@pytest.mark.parametrize("case", ["plain", "dead", "spike", "dead_last", "dead_first_spike"])
def test_oracle_surface_wave_prep_matches_reference(case):
    from oracle import preprocess as op
    g = gio.load("prep")
    for m in ("surface_wave", "xcorr"):
        o = op.surface_wave_prep(g[case + "_in"].astype(np.float64), float(g["dt"]), method=m)
        assert np.abs(o - g[f"{case}_{m}"]).max() <= 1e-12 * np.abs(g[f"{case}_{m}"]).max()


SELECT_CASES = ["default", "short", "odd", "spacing"]


@pytest.mark.parametrize("case", SELECT_CASES)
def test_oracle_window_selection_matches_reference(case):
    """oracle.select.locate_windows vs SurfaceWaveSelector (apis/data_classes.py:170-223) run in the
    survey container: accepted passes, slice bounds and the cut data's sums."""
    from oracle import select as osel
    g = gio.load("select")
    c = gio.select_cases()[case]
    t_axis = c["t_axis"]
    got = osel.locate_windows(t_axis.size, t_axis, c["dist"], c["x0"], c["start_x_tracking"], c["veh_states"],
                              c["t_trk"], t_axis[1] - t_axis[0], **c["kw"])
    ref = g[case + "_windows"]
    n_t = c["rec"].shape[1]
    assert [(k, sx, ex, st, min(et, n_t)) for k, sx, ex, st, et in got] == [tuple(r) for r in ref.tolist()]
    sums = [np.array(c["rec"][sx:ex, st:et]).sum() for _, sx, ex, st, et in got]
    assert np.array_equal(np.array(sums), g[case + "_sums"])
    vx = [osel.veh_state_xt(c["veh_states"][k], c["start_x_tracking"], c["dist_trk"], c["t_trk"]) for k, *_ in got]
    if vx:
        assert np.array_equal(np.concatenate([v[0] for v in vx]), g[case + "_vx"])
        assert np.array_equal(np.concatenate([v[1] for v in vx]), g[case + "_vt"])


def test_oracle_daily_xcorr_workflow_matches_reference():
    """The xcorr flavour of the daily workflow restated with the oracle (apis/imaging_workflow.py:33-80, 199-201):
    per record the xcorr preprocessing, the window selection, VirtualShotGather per window (norm=False, two-sided)
    and the class mean; the day's image as the sum of per-record means, against tests/golden/workflow.npz; then
    compute_disp_image() with its defaults (whole gather, norm=False)."""
    from oracle import disp as odisp
    from oracle import preprocess as op
    from oracle import select as osel
    from oracle import vsg as ovsg
    g = gio.load("workflow")
    day = None
    for k, c in enumerate(gio.workflow_files()):
        t_axis = c["t_axis"]
        d = op.surface_wave_prep(c["rec"], t_axis[1] - t_axis[0], method="xcorr", scipy_filter=True)
        dist = (c["x_axis"] - 400) * 8.16
        wins = osel.locate_windows(t_axis.size, t_axis, dist, c["x0"], c["start_x_tracking"], c["veh_states"],
                                   c["t_trk"], t_axis[1] - t_axis[0], **c["select_kw"])
        assert len(wins) == int(g[f"n_windows_{k}"])
        kw = dict(c["imaging_kw"])
        other = kw.pop("include_other_side")
        gathers = []
        for kv, sx, ex, st, et in wins:
            vx, vt = osel.veh_state_xt(c["veh_states"][kv], c["start_x_tracking"], c["dist_trk"], c["t_trk"])
            w = dict(data=d[sx:ex, st:et], x_axis=dist[sx:ex], t_axis=t_axis[st:et], veh_state_x=vx, veh_state_t=vt)
            gathers.append(ovsg.virtual_shot_gather(w, include_other_side=other, norm=False, **kw))
        assert [x[0].shape[-1] for x in gathers] == list(g[f"w_{k}"])
        mean = ovsg.stack([x[0] for x in gathers])
        assert np.abs(mean - g[f"file_avg_{k}"]).max() <= 1e-9 * np.abs(g[f"file_avg_{k}"]).max()
        if day is None:
            day, gx, gt = mean, gathers[0][1], gathers[0][2]
        else:
            n = min(day.shape[-1], mean.shape[-1])
            day = day.copy()
            day[:, :n] += mean[:, :n]
    assert np.abs(day - g["day_xcf"]).max() <= 1e-9 * np.abs(g["day_xcf"]).max()
    assert np.array_equal(gx, g["day_x_axis"]) and np.array_equal(gt, g["day_t_axis"])
    fv = odisp.compute_disp_image(day, gx, gt)
    assert np.abs(fv - g["day_fv"]).max() <= 1e-6 * np.abs(g["day_fv"]).max()
