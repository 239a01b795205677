"""More GPU parity of the fused correlate-and-stack path: passes whose pivot sits at different gather
rows within one launch (odd row count), and windows the reference turns into NaN gathers
(data / ||data||_F with a NaN, apis/virtual_shot_gather.py:125)."""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4
KW = dict(pivot=700, start_x=500, end_x=900, wlen=2)


def _fixture_batch(device, name="vsg_w500", **kw):
    import torch

    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry
    g = gio.load(name)
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(gio.n_pass(g))]
    prm = VsgParams(**{**KW, **kw})
    geoms = [pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, prm) for w in wins]
    data = torch.as_tensor(np.stack([w.data for w in wins]), device=device)
    return g, wins, prm, VsgPlan(geoms, prm, data.shape[1], data.shape[2]), data


def _mixed_batch(device, n_each=12, seed=5, t0=None):
    """Passes generated at two fiber offsets: the pivot is gather row 24 for one half, 25 for the
    other (R = 49 for both), so shared and trajectory rows differ between passes of one launch."""
    import torch

    from das_diff_veh_amd.synth import DT_W500, synth_batch_device
    out = []
    for off in (0.0, 4.0):
        w, x, t, trk, _ = synth_batch_device(n_each, pivot=700.0, seed=seed + int(off), device=device,
                                             x_first=700 - 30 * 8.16 + off, t0=DT_W500 if t0 is None else t0)
        out.append((w, x, t, trk))
    wins = torch.cat([o[0] for o in out])
    xs = [o[1] for o in out for _ in range(n_each)]
    ts = [o[2] for o in out for _ in range(n_each)]
    trk = [tr for o in out for tr in o[3]]
    return wins, xs, ts, trk


@pytest.mark.parametrize("w", [500, 499])
@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True),
                                dict(include_other_side=False, norm=False)])
def test_stack_mixed_pivot_rows(device, kw, w):
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry
    from das_diff_veh_amd.synth import DT_W499, DT_W500
    from oracle import vsg as ovsg
    wins, xs, ts, trk = _mixed_batch(device, t0=DT_W500 if w == 500 else DT_W499)
    prm = VsgParams(**{**KW, **kw})
    geoms = [pass_geometry(x, t, vx, vt, prm) for x, t, (vx, vt) in zip(xs, ts, trk)]
    assert {g.pivot_idx - g.start_idx for g in geoms} == {24, 25} and {g.end_idx - g.start_idx for g in geoms} == {49}
    assert geoms[0].w == w
    plan = VsgPlan(geoms, prm, wins.shape[1], wins.shape[2])
    slots = np.arange(len(geoms)) % 3
    sched = vsg.StackSchedule(slots, 3, chunk=4)
    got = vsg.vsg_stack(wins, plan, sched).double().cpu().numpy()
    host = wins.double().cpu().numpy()
    for s in range(3):
        refs = []
        for i in np.flatnonzero(slots == s):
            o = dict(data=host[i], x_axis=xs[i], t_axis=ts[i], veh_state_x=trk[i][0], veh_state_t=trk[i][1])
            refs.append(ovsg.virtual_shot_gather(o, **kw, **KW)[0])
        assert gio.gather_rel_err(got[s], ovsg.stack(refs)) < TOL, (s, kw)


def test_stack_invalid_windows(device):
    """A NaN anywhere in a window makes that pass's whole gather NaN (the reference divides by
    ||data||_F, apis/virtual_shot_gather.py:125); a zeroed channel drops out exactly."""
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import VsgPlan
    from oracle import vsg as ovsg
    g, wins, prm, plan, data = _fixture_batch(device, include_other_side=True, norm=False)
    geo = plan.geoms[0]
    a, L = geo.seg[0, 0]
    data = data.clone()
    data[0, geo.start_idx + 2, a + 10] = float("nan")
    data[1, geo.start_idx + 4] = 0.0
    host = data.double().cpu().numpy()
    refs = []
    for i in range(plan.n_pass):
        p1 = VsgPlan([plan.geoms[i]], prm, plan.n_ch, plan.n_t)
        got = vsg.vsg_stack(data[i:i + 1], p1, vsg.StackSchedule(np.zeros(1, np.int64), 1, chunk=1))
        o = gio.oracle_window(g, i)
        o["data"] = host[i]
        with np.errstate(all="ignore"):
            refs.append(ovsg.virtual_shot_gather(o, include_other_side=True, norm=False, **KW)[0])
        assert gio.gather_rel_err(got.double().cpu().numpy()[0], refs[i]) < TOL, i
    got = vsg.vsg_stack(data, plan, vsg.StackSchedule(np.zeros(plan.n_pass, np.int64), 1, chunk=2))
    with np.errstate(all="ignore"):
        assert gio.gather_rel_err(got.double().cpu().numpy()[0], ovsg.stack(refs)) < TOL


def test_skip_failed_passes_stack_the_rest(device):
    """get_images(skip_failed=True): the broken passes are reported, the class mean is that of the
    imaged passes (golden gathers 0 and 3), and without the flag the list raises like the reference."""
    from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows
    from oracle import vsg as ovsg
    from tests.test_host import _failing_windows
    wins, g = _failing_windows()
    imgs = VirtualShotGathersFromWindows(wins)
    imgs.get_images(include_other_side=True, pivot=700, start_x=500, end_x=900, wlen=2, skip_failed=True)
    assert sorted(imgs.failed) == [1, 2, 3]
    ref = ovsg.stack([g["xcf"][0], g["xcf"][3]])
    assert gio.gather_rel_err(imgs.avg_image.XCF_out, ref) < 1e-4
    assert len(imgs.images) == 2
    with pytest.raises(ValueError):
        VirtualShotGathersFromWindows(wins).get_images(include_other_side=True, pivot=700, start_x=500, end_x=900,
                                                       wlen=2)


@pytest.mark.parametrize("w", [500, 499])
@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True),
                                dict(include_other_side=False, norm=False)])
def test_pivot_table_matches_per_subwindow_transforms(device, kw, w):
    """The stack launch with the per-pass pivot-slice spectra table (receivers two per transform) equals the
    per-sub-window transforms (z = pivot + i receiver) on mixed pivot rows and on configs[2]-like far rows
    (trajectory windows clamped to [0, nsamp): the table's far-row entries)."""
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry
    from das_diff_veh_amd.synth import DT_W499, DT_W500, synth_batch_device
    t0 = DT_W500 if w == 500 else DT_W499
    wins, xs, ts, trk = _mixed_batch(device, t0=t0)
    prm = VsgParams(**{**KW, **kw})
    geoms = [pass_geometry(x, t, vx, vt, prm) for x, t, (vx, vt) in zip(xs, ts, trk)]
    assert geoms[0].w == w
    cases = [(wins, VsgPlan(geoms, prm, wins.shape[1], wins.shape[2]))]
    w_, x, t, trk2, _ = synth_batch_device(6, n_ch=256, n_t=4096, pivot=1044.0, seed=31, device=device, x_first=0.0,
                                           track_half=300, chunk=2, t0=t0)
    prm2 = VsgParams(pivot=1044.0, start_x=0.0, end_x=2100.0, wlen=2, **kw)
    geoms2 = [pass_geometry(x, t, vx, vt, prm2) for vx, vt in trk2]
    cases.append((w_, VsgPlan(geoms2, prm2, w_.shape[1], w_.shape[2])))
    for wins_c, plan in cases:
        slots = np.arange(plan.n_pass) % 2
        sched = vsg.StackSchedule(slots, 2, chunk=4)
        sc = vsg.vsg_scales(wins_c, plan)
        a = vsg.vsg_stack(wins_c, plan, sched, scales=sc, table=True).double().cpu().numpy()
        b = vsg.vsg_stack(wins_c, plan, sched, scales=sc, table=False).double().cpu().numpy()
        assert np.array_equal(np.isnan(a), np.isnan(b))
        m = np.isfinite(a)
        for s in range(2):
            assert gio.gather_rel_err(np.where(m[s], a[s], 0.0), np.where(m[s], b[s], 0.0)) < 1e-5, (s, kw)


@pytest.mark.parametrize("twin", [5, 6])
@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True),
                                dict(include_other_side=False, norm=False)])
def test_long_xcorr_window_stack(device, twin, kw):
    """time_window_to_xcorr = 5 / 6 at w = 500 gives nwin = 4 / 5 sub-windows per side, more than the pivot-slice
    table's entries hold (3): such passes are marked unusable by the table kernel and take the plain
    per-sub-window path.  Stack with and without the table, and the validated launch, equal the oracle."""
    from das_diff_veh_amd import vsg
    from oracle import vsg as ovsg
    g, wins, prm, plan, data = _fixture_batch(device, time_window_to_xcorr=twin, **kw)
    assert plan.w == 500 and int(twin / 0.003999999999997783) >= 1250
    slots = np.arange(plan.n_pass) % 2
    sched = vsg.StackSchedule(slots, 2, chunk=2)
    sc = vsg.vsg_scales(data, plan)
    a = vsg.vsg_stack(data, plan, sched, scales=sc, table=True).double().cpu().numpy()
    b = vsg.vsg_stack(data, plan, sched, scales=sc, table=False).double().cpu().numpy()
    host = data.double().cpu().numpy()
    for s in range(2):
        refs = []
        for i in np.flatnonzero(slots == s):
            o = gio.oracle_window(g, i)
            o["data"] = host[i]
            refs.append(ovsg.virtual_shot_gather(o, time_window_to_xcorr=twin, **kw, **KW)[0])
        ref = ovsg.stack(refs)
        assert gio.gather_rel_err(a[s], ref) < TOL, (s, twin, kw)
        assert gio.gather_rel_err(b[s], ref) < TOL, (s, twin, kw)
    if plan.flags & 6:
        v = vsg.vsg_stack_validated(data, plan, sched, scales=vsg.vsg_scales(data, plan, validity=False))
        v = v.double().cpu().numpy()
        assert np.array_equal(np.isnan(v), np.isnan(a))  # rows the reference leaves NaN (0 / 0 norms)
        m = np.isfinite(a)
        assert np.allclose(v[m], a[m], rtol=0, atol=1e-6 * np.abs(a[m]).max())

