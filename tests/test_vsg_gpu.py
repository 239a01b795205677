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


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
@pytest.mark.parametrize("kw", [
    dict(include_other_side=True, norm=False),
    dict(include_other_side=True),
    dict(include_other_side=False),
    dict(include_other_side=True, norm=False, norm_amp=False),
    dict(include_other_side=False, norm=False),
])
@pytest.mark.parametrize("special", [False, True])
def test_stack_modes(device, fixture, kw, special):
    """Fused correlate-and-stack for every flag combination, two classes, against the oracle.
    With ``special`` passes get half their channels zeroed (one side of the gather is 0/0 and must
    drop out of the two-sided average), all channels zeroed, or a NaN sample, which must propagate
    exactly as sum(images)/len(images) does in the reference (imaging_classes.py:127)."""
    from das_diff_veh_amd import engine
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.plan import VsgParams
    from oracle import vsg as ovsg
    g = gio.load(fixture)
    n = gio.n_pass(g)
    arrs = [gio.pass_arrays(g, i) for i in range(n)]
    if special:
        for i, kind in zip(range(n), ["low", "high", "zero", "nan"]):
            d = arrs[i]["data"].copy()
            half = d.shape[0] // 2
            if kind == "low":
                d[:half] = 0
            elif kind == "high":
                d[half:] = 0
            elif kind == "zero":
                d[:] = 0
            else:
                d[5, 1000] = np.nan
            arrs[i]["data"] = d
    wins = [SurfaceWaveWindow(**a) for a in arrs]
    slots = np.array([i % 2 for i in range(n)])
    prm = VsgParams(**kw, **KW)
    got, _ = engine.stacked(wins, prm, slots=slots, n_slot=2, device=device, chunk=2)
    got = got.double().cpu().numpy()
    for s in range(2):
        refs = []
        for i in np.where(slots == s)[0]:
            o = gio.oracle_window(g, i)
            o["data"] = arrs[i]["data"].astype(np.float64)
            with np.errstate(all="ignore"):
                refs.append(ovsg.virtual_shot_gather(o, **kw, **KW)[0])
        with np.errstate(all="ignore"):
            ref = ovsg.stack(refs)
        assert gio.gather_rel_err(got[s], ref) < TOL, (s, kw)


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
@pytest.mark.parametrize("kind", ["zero", "nan", "inf", "nan_outside_rows", "inf_in_slice", "nan_in_slice",
                                  "nan_direct", "nan_zero_pivot"])
def test_validated_stack_invalid_windows(device, kind, fixture):
    """vsg_stack_validated: an all-zero window, or a NaN / inf anywhere in it (also in channels no gather
    row reads), makes its class mean NaN (data / ||data||_F, apis/virtual_shot_gather.py:125); the
    other class is unaffected and equals the oracle.  The slice cases put the sample where the covered-span scan
    leaves it to the correlation: a trajectory row's slice (P + i R transforms), a one-sided row below the pivot
    (its receivers packed across passes: the task's non-finite sum sends its passes to the whole-window rescan),
    and the same with the pivot's slices zeroed (a sub-window never transformed, checked where it is loaded)."""
    import torch

    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.engine import group_windows
    from das_diff_veh_amd.plan import VsgParams
    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack_validated
    from oracle import vsg as ovsg
    g = gio.load(fixture)
    n = gio.n_pass(g)
    arrs = [gio.pass_arrays(g, i) for i in range(n)]
    d = arrs[1]["data"].copy()
    if kind == "zero":
        d[:] = 0
    elif kind == "nan":
        d[10, 2000] = np.nan
    elif kind == "inf":
        d[30, 100] = np.inf
    elif kind == "nan_outside_rows":
        d[-1, -1] = np.nan  # the last channel is beyond end_x: no gather row reads it
    else:  # inside a forward-side correlation slice of a gather row (checked by the correlation wave)
        from das_diff_veh_amd.plan import pass_geometry
        a = arrs[1]
        w0 = SurfaceWaveWindow(**a)
        geo = pass_geometry(a["x_axis"], a["t_axis"], w0.veh_state_x, w0.veh_state_t,
                            VsgParams(include_other_side=True, norm=False, **KW))
        below = kind in ("nan_direct", "nan_zero_pivot")
        i = geo.pivot_idx - geo.start_idx + (-3 if below else 3)
        t0, L = geo.seg[i, 0]
        assert L == geo.nsamp and L > 400  # a full-length slice (nsamp = 1000 at w = 500, 999 at w = 499)
        d[geo.start_idx + i, t0 + 400] = np.inf if kind == "inf_in_slice" else np.nan
        if kind == "nan_zero_pivot":  # the pivot's forward window (the shared slices of the rows below it)
            tp, Lp = geo.seg[geo.pivot_idx - geo.start_idx, 0]
            d[geo.pivot_idx, tp:tp + Lp] = 0
    arrs[1]["data"] = d
    wins = [SurfaceWaveWindow(**a) for a in arrs]
    two = kind not in ("nan_direct", "nan_zero_pivot")  # one-sided rows below the pivot: cross-pass packed tasks
    prm = VsgParams(include_other_side=two, norm=False, **KW)
    (idx, plan), = group_windows(wins, prm, device)[0]
    data = torch.as_tensor(np.stack([w.data for w in wins]), dtype=torch.float32, device=device)
    slots = np.array([i % 2 for i in range(n)])
    got = vsg_stack_validated(data, plan, StackSchedule(slots[idx], 2, chunk=2)).double().cpu().numpy()
    assert plan.w == (500 if fixture == "vsg_w500" else 499)
    assert np.isnan(got[1]).all()
    refs = [ovsg.virtual_shot_gather(gio.oracle_window(g, i), include_other_side=two, norm=False, **KW)[0]
            for i in range(n) if slots[i] == 0]
    assert gio.gather_rel_err(got[0], ovsg.stack(refs)) < TOL


@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True),
                                dict(include_other_side=False, norm=False)])
def test_validated_stack_w499(device, kw):
    """w = 499 (the reference's dt = 0.004000000000001336 operating point): the fused validated launch (padded
    1 024-point transforms, frequency-domain class sums, the validity scan in the same launch) equals the
    oracle's class means, with chunks of 1 (every pass its own task) and of 3."""
    import torch

    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.engine import group_windows
    from das_diff_veh_amd.plan import VsgParams
    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack_validated
    from oracle import vsg as ovsg
    g = gio.load("vsg_w499")
    n = gio.n_pass(g)
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(n)]
    prm = VsgParams(**kw, **KW)
    if not (prm.flags & 6):
        pytest.skip("validated stacking needs norm or norm_amp")
    (idx, plan), = group_windows(wins, prm, device)[0]
    assert plan.w == 499
    data = torch.as_tensor(np.stack([w.data for w in wins]), dtype=torch.float32, device=device)
    slots = np.array([i % 2 for i in range(n)])
    refs = [[ovsg.virtual_shot_gather(gio.oracle_window(g, i), **kw, **KW)[0] for i in range(n) if slots[i] == s]
            for s in range(2)]
    for chunk in (1, 3):
        got = vsg_stack_validated(data, plan, StackSchedule(slots[idx], 2, chunk=chunk)).double().cpu().numpy()
        for s in range(2):
            assert gio.gather_rel_err(got[s], ovsg.stack(refs[s])) < TOL, (s, chunk, kw)
