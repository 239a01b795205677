"""Device-derived index tables (dvh_pass_geometry) equal the host restatement pass_geometry bit for bit.

pass_geometry (das_diff_veh_amd/plan.py) is itself checked against the reference's slices in
tests/test_host.py; here the kernel must reproduce it exactly over the golden windows, the synth10k
geometry of BASELINE configs[2] (R = 1023, most rows' trajectory times outside the window ->
argmax = 0 reads), early / late / slow passes and per-pass axes.
"""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu


def _compare(x_axis, t_axis, trks, prm, n_ch, device, pivot_x=None):
    from das_diff_veh_amd.plan import DevicePlan, VsgPlan, pack_trajectories, pass_geometry
    xs = x_axis if np.ndim(x_axis) == 2 else [x_axis] * len(trks)
    ts = t_axis if np.ndim(t_axis) == 2 else [t_axis] * len(trks)
    geoms = [pass_geometry(x, t, vx, vt, prm) for x, t, (vx, vt) in zip(xs, ts, trks)]
    host = VsgPlan(geoms, prm, n_ch, len(ts[0]))
    tx, tt, tl = pack_trajectories(trks, device)
    dev = DevicePlan(x_axis, t_axis, tx, tt, tl, prm, n_ch, pivot_x=pivot_x).check()
    assert (dev.R, dev.w, dev.hop, dev.nsamp) == (host.R, host.w, host.hop, host.nsamp)
    assert np.array_equal(dev.pass_tab.cpu().numpy(), host.pass_tab)
    got = dev.host_seg_tab()
    if not np.array_equal(got, host.seg_tab):
        bad = np.argwhere(got != host.seg_tab)[:5]
        raise AssertionError(f"seg_tab differs at {bad.tolist()}: {got[tuple(bad[0])]} vs {host.seg_tab[tuple(bad[0])]}")
    assert dev.algorithmic_bytes(3) == host.algorithmic_bytes(3)
    return host


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
@pytest.mark.parametrize("other", [True, False])
def test_golden_windows(device, fixture, other):
    from das_diff_veh_amd.plan import VsgParams
    g = gio.load(fixture)
    ws = [gio.oracle_window(g, i) for i in range(gio.n_pass(g))]
    prm = VsgParams(pivot=700, start_x=500, end_x=900, wlen=2, include_other_side=other)
    _compare(np.stack([w["x_axis"] for w in ws]), np.stack([w["t_axis"] for w in ws]),
             [(w["veh_state_x"], w["veh_state_t"]) for w in ws], prm, ws[0]["data"].shape[0], device)


@pytest.mark.parametrize("case", ["early", "late", "slow", "p680", "narrow", "wlen1"])
def test_edge_windows(device, case):
    import ast

    from das_diff_veh_amd.plan import VsgParams
    g = gio.load("vsg_edge")
    w = gio.oracle_window(g, 0, prefix=case + "_")
    kw = ast.literal_eval(str(g[case + "_kw"]))
    prm = VsgParams(include_other_side=True, norm=False, **kw)
    _compare(w["x_axis"], w["t_axis"], [(w["veh_state_x"], w["veh_state_t"])], prm, w["data"].shape[0], device)


def synth10k_trajectories(x_axis, t_axis, seed, n):
    """n - 2 regular passes: a slow (15 m/s) and a fast (30 m/s) one whose far rows leave the window,
    then bench-style ones (15-30 m/s, crossing the pivot within +-1 s of mid-window); and 2 edge passes
    last: crossing 0.5 s after the window start (other-side shared slice empty: pt - nsamp < 0 wraps,
    so that side's pivot row is 0 and its rows are x / 0 = +-inf in the reference) and 2 s before its
    end (forward shared slice shorter than one sub-window: the forward side is +-inf / NaN)."""
    from das_diff_veh_amd.synth import TRACK_DT
    rng = np.random.default_rng(seed)
    xs = np.arange(np.floor(4178.0) - 4300, np.floor(4178.0) + 4301, 1.0)
    T = t_axis.size
    specs = [(15.0, t_axis[T // 2]), (30.0, t_axis[T // 2] + 0.3)]
    specs += [(rng.uniform(15, 30), t_axis[T // 2] + rng.uniform(-1, 1)) for _ in range(max(n - 4, 0))]
    specs = specs[:max(n - 2, 0)] + [(22.0, t_axis[0] + 0.5), (18.0, t_axis[-1] - 2.0)][:n]
    return [(xs, np.round((tc + (xs - 4178.0) / v) / TRACK_DT) * TRACK_DT) for v, tc in specs[:n]]


def test_synth10k_geometry(device):
    from das_diff_veh_amd.plan import VsgParams
    from das_diff_veh_amd.synth import DT_W500
    x_axis = 0.37 + 8.16 * np.arange(1024)
    t_axis = DT_W500 + np.arange(8192) * 0.004
    prm = VsgParams(pivot=4178.0, start_x=0.0, end_x=8400.0, wlen=2, norm=False, include_other_side=True)
    trks = synth10k_trajectories(x_axis, t_axis, 11, 64)
    host = _compare(x_axis, t_axis, trks, prm, 1024, device)
    assert host.R == 1023
    # the reference's "trajectory time beyond the window -> argmax = 0 -> read [0, nsamp)" quirk is
    # exercised on most rows
    f_beyond = sum(int(np.sum(np.interp(x_axis, vx, vt) + 1 > t_axis[-1])) for vx, vt in trks)
    assert f_beyond > 1000


def test_bad_trajectory_status(device):
    import torch

    from das_diff_veh_amd.plan import DevicePlan, VsgParams, pack_trajectories
    g = gio.load("vsg_w500")
    w = gio.oracle_window(g, 0)
    vx, vt = w["veh_state_x"], w["veh_state_t"]
    # reversed: sorted like interp1d's mergesort -> the same tables; a repeated abscissa (interp1d would
    # divide by zero) and a single point (interp1d raises) are flagged
    trks = [(vx, vt), (vx[::-1], vt[::-1]), (np.r_[vx[:5], vx[4:]], np.r_[vt[:5], vt[4:]]), (vx[:1], vt[:1])]
    tx, tt, tl = pack_trajectories(trks, device)
    dev = DevicePlan(w["x_axis"], w["t_axis"], tx, tt, tl, VsgParams(pivot=700, start_x=500, end_x=900),
                     w["data"].shape[0])
    torch.cuda.synchronize()
    assert dev.status.cpu().numpy().tolist() == [0, 0, 1, 1]
    seg = dev.host_seg_tab()
    assert np.array_equal(seg[0], seg[1])
    with pytest.raises(ValueError):
        dev.check()


def test_host_trajectory_status_equals_kernel(device):
    """pack_trajectories_checked's host status (engine.stacked's check without a device round trip) equals the
    geometry kernel's on sorted, reversed, repeated, NaN, single-point and empty trajectories."""
    import torch

    from das_diff_veh_amd.plan import DevicePlan, VsgParams, pack_trajectories_checked
    g = gio.load("vsg_w500")
    w = gio.oracle_window(g, 0)
    vx, vt = w["veh_state_x"], w["veh_state_t"]
    nan_x = vx.copy()
    nan_x[7] = np.nan
    shuffled = np.random.default_rng(1).permutation(vx.size)
    trks = [(vx, vt), (vx[::-1], vt[::-1]), (np.r_[vx[:5], vx[4:]], np.r_[vt[:5], vt[4:]]), (vx[:1], vt[:1]),
            (nan_x, vt), (vx[shuffled], vt[shuffled]), (vx[:0], vt[:0]), (vx[:2], vt[:2]), (vx[[1, 1]], vt[:2])]
    (tx, tt, tl), bad = pack_trajectories_checked(trks, device)
    dev = DevicePlan(w["x_axis"], w["t_axis"], tx, tt, tl, VsgParams(pivot=700, start_x=500, end_x=900),
                     w["data"].shape[0])
    torch.cuda.synchronize()
    assert bad.tolist() == dev.status.cpu().numpy().tolist() == [0, 0, 1, 1, 1, 0, 1, 0, 1]
    with pytest.raises(ValueError):
        dev.check(bad)
    assert dev.check(np.zeros(len(trks), np.int32)) is dev


@pytest.mark.parametrize("seed,npts", [(3, 400), (4, 1500)])  # 1500: beyond the kernel's LDS-staged trajectories
def test_irregular_axes_geometry(device, seed, npts):
    """Non-uniform t axes (jittered steps, a 20x-denser stretch, repeated samples) and trajectories
    with uneven abscissa spacing, so the kernel's guessed search misses its first guess on both sides
    and falls back to the narrowed bisection; the tables must still equal the host's."""
    from das_diff_veh_amd.plan import VsgParams
    rng = np.random.default_rng(seed)
    n_pass, T = 12, 4096
    from das_diff_veh_amd.synth import DT_W500
    x_axis = np.sort(rng.uniform(0.0, 2000.0, size=256))
    steps = 0.004 * rng.uniform(0.2, 1.8, size=(n_pass, T))
    steps[:, 1000:1600] *= 0.05
    steps[:, 2000:2010] = 0.0
    # the first step sets dt (and w, nsamp) as in the reference: keep it the bench's exact 0.004
    t_axis = np.empty((n_pass, T))
    t_axis[:, :2] = DT_W500 + np.arange(2) * 0.004
    t_axis[:, 2:] = t_axis[:, 1:2] + np.cumsum(steps[:, 2:], axis=1)
    trks = []
    for p in range(n_pass):
        xs = np.sort(rng.choice(np.arange(-200.0, 2200.0, 0.5), size=npts, replace=False))
        v = rng.uniform(12.0, 30.0)
        tc = t_axis[p, rng.integers(T // 4, 3 * T // 4)]
        trks.append((xs, tc + (xs - 1000.0) / v + 0.05 * np.sin(xs / 37.0)))
    prm = VsgParams(pivot=1000.0, start_x=300.0, end_x=1700.0, wlen=2, norm=False, include_other_side=True)
    _compare(x_axis, t_axis, trks, prm, 256, device)


def test_plan_slices_share_one_derive(device):
    """DevicePlan.slice: one derive() of the whole plan gives every slice the tables its own
    derive() forms (the bench derives a step's batches in one launch)."""
    import torch

    from das_diff_veh_amd.plan import DevicePlan, VsgParams, pack_trajectories
    from das_diff_veh_amd.synth import DT_W500
    x_axis = 0.37 + 8.16 * np.arange(1024)
    t_axis = DT_W500 + np.arange(8192) * 0.004
    prm = VsgParams(pivot=4178.0, start_x=0.0, end_x=8400.0, wlen=2, norm=False, include_other_side=True)
    trks = synth10k_trajectories(x_axis, t_axis, 5, 37)
    tx, tt, tl = pack_trajectories(trks, device)
    whole = DevicePlan(x_axis, t_axis, tx, tt, tl, prm, 1024).check()
    ref = whole.host_seg_tab().copy()
    parts = [whole.slice(a, min(a + 16, 37)) for a in range(0, 37, 16)]
    whole.seg_tab.fill_(-1)
    whole.derive()
    torch.cuda.synchronize()
    assert np.array_equal(np.concatenate([p.host_seg_tab() for p in parts]), ref)
    whole.seg_tab.fill_(-1)
    for p in parts:
        p.derive()
    torch.cuda.synchronize()
    assert np.array_equal(whole.host_seg_tab(), ref)
    assert [p.n_pass for p in parts] == [16, 16, 5]
    assert np.array_equal(parts[1].pass_tab.cpu().numpy(), whole.pass_tab.cpu().numpy()[16:32])
    with pytest.raises(ValueError):
        whole.slice(30, 40)
