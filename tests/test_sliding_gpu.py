"""GPU parity of sliding-pivot launches: one launch images every
(pass, pivot) unit, pivots every 8 channels with start_x / end_x = pivot -/+ 200 m, each unit
checked against the oracle's VirtualShotGather at that pivot (apis/virtual_shot_gather.py:183-192)."""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _case(device, n=3, n_ch=300, n_t=8192, seed=11):
    from das_diff_veh_amd.synth import synth_batch_device
    w, x, t, trk, _ = synth_batch_device(n, n_ch=n_ch, n_t=n_t, pivot=1224.0, seed=seed, device=device,
                                         x_first=0.37, track_half=1500, chunk=1)
    return w, x, t, trk


def _oracle_unit(host, x, t, trk, plan, u, kw):
    from oracle import vsg as ovsg
    q, j = int(plan.unit_window[u]), int(plan.unit_pivot[u])
    p = float(x[plan.pivots[j]])
    o = dict(data=host[q], x_axis=x, t_axis=t, veh_state_x=trk[q][0], veh_state_t=trk[q][1])
    return ovsg.virtual_shot_gather(o, pivot=p, start_x=p - 200.0, end_x=p + 200.0, wlen=2, **kw)[0]


@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True),
                                dict(include_other_side=False, norm=False)])
def test_sliding_unit_gathers(device, kw):
    _check_gathers(device, kw, full_only=True, n=8)


@pytest.mark.parametrize("kw", [dict(include_other_side=True, norm=False), dict(include_other_side=True)])
def test_sliding_all_pivots(device, kw):
    """Every pivot, including those whose trajectory slices leave the window (short / empty
    sub-window sets, all-zero sides -> the reference's zeros and 0/0 NaNs)."""
    _check_gathers(device, kw, full_only=False, n=3)


def _check_gathers(device, kw, full_only, n):
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    w, x, t, trk = _case(device, n=n)
    prm = VsgParams(**kw)
    pch = np.arange(32, w.shape[1] - 32, 8)
    plan = UnitPlan.sliding(x, t, trk, pch, 200.0, prm, full_only=full_only)
    assert plan.n_pass >= (6 if full_only else n * len(pch))
    flat = vsg.flat_units(w, plan)
    sc = vsg.vsg_scales(flat, plan, win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan))
    got = vsg.vsg_gathers(flat, plan, sc).double().cpu().numpy()
    host = w.double().cpu().numpy()
    finite_scale = np.isfinite(sc.cpu().numpy()).all(axis=1)
    for u in range(plan.n_pass):
        with np.errstate(all="ignore"):
            ref = _oracle_unit(host, x, t, trk, plan, u, kw)
        if finite_scale[u]:
            assert gio.gather_rel_err(got[u], ref) < TOL, (u, kw)
        else:
            # a side whose pivot slice is empty (Python-slice wrap at the window start) has
            # amax(pivot row) = 0: the reference's x / 0 gives +-inf with the sign of x, and for
            # correlations that are 0 up to rounding that sign is rounding noise (fp32 vs float64),
            # so only the finite / NaN / inf positions are compared
            assert not full_only
            assert np.array_equal(np.isnan(got[u]), np.isnan(ref)) and np.array_equal(np.isinf(got[u]), np.isinf(ref))
            m = np.isfinite(ref)
            assert gio.gather_rel_err(np.where(m, got[u], 0.0), np.where(m, ref, 0.0)) < TOL, u


def test_sliding_class_stacks(device):
    """Per-(class, pivot) stacks of one launch == the oracle's mean of that pivot's unit gathers."""
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    from oracle import vsg as ovsg
    w, x, t, trk = _case(device, n=4, seed=12)
    kw = dict(include_other_side=True, norm=False)
    pch = np.arange(32, w.shape[1] - 32, 8)
    plan = UnitPlan.sliding(x, t, trk, pch, 200.0, VsgParams(**kw))
    cls = plan.unit_window % 2
    slots = cls * len(pch) + plan.unit_pivot
    n_slot = 2 * len(pch)
    flat = vsg.flat_units(w, plan)
    sched = vsg.StackSchedule(slots, n_slot, chunk=2)
    got = vsg.vsg_stack(flat, plan, sched, win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan))
    got = got.double().cpu().numpy()
    host = w.double().cpu().numpy()
    checked = 0
    for s in np.unique(slots):
        units = np.flatnonzero(slots == s)
        ref = ovsg.stack([_oracle_unit(host, x, t, trk, plan, u, kw) for u in units])
        assert gio.gather_rel_err(got[s], ref) < TOL, s
        checked += 1
    empty = np.setdiff1d(np.arange(n_slot), slots)
    assert np.all(got[empty] == 0.0) and checked >= 4


def test_sliding_at_scale_flattened_offsets(device):
    """configs[3] geometry at scale: 72 windows x 4096 channels x 8192 samples as ONE flattened
    [72 * 4096, 8192] record, so the units' q * C row offsets pass 2^18 (up to 71 * 4096 = 290,816);
    trajectories as the sliding bench draws them (crossing uniform along the fiber, 15-30 m/s).
    Units of the first two and the last four windows are checked against the oracle."""
    import torch

    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    from das_diff_veh_amd.synth import TRACK_DT, synth_batch_device
    n, C, T = 72, 4096, 8192
    w, x, t, _, _ = synth_batch_device(n, n_ch=C, n_t=T, pivot=C * 8.16 / 2, seed=21, device=device, x_first=0.37,
                                       track_half=10, chunk=2)
    rng = np.random.default_rng(5)
    trk = []
    for xa, va, ta in zip(rng.uniform(x[32], x[-32], n), rng.uniform(15.0, 30.0, n),
                          t[T // 2] + rng.uniform(-1.0, 1.0, n)):
        xs = np.arange(np.floor(xa) - 800.0, np.floor(xa) + 801.0)
        trk.append((xs, np.round((ta + (xs - xa) / va) / TRACK_DT) * TRACK_DT))
    kw = dict(include_other_side=True, norm=False)
    pch = np.arange(32, C - 32, 8)
    plan = UnitPlan.sliding(x, t, trk, pch, 200.0, VsgParams(**kw))
    assert int(plan.pass_tab[:, 1].max()) > 2 ** 18
    flat = vsg.flat_units(w, plan)
    sc = vsg.vsg_scales(flat, plan, win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan))
    got = vsg.vsg_gathers(flat, plan, sc)
    check = np.flatnonzero((plan.unit_window < 2) | (plan.unit_window >= n - 4))
    assert check.size >= 6 and int(plan.unit_window[check].max()) == n - 1
    hosts = {}
    for u in check:
        q = int(plan.unit_window[u])
        if q not in hosts:
            hosts[q] = w[q].double().cpu().numpy()
        j = int(plan.unit_pivot[u])
        p = float(x[plan.pivots[j]])
        from oracle import vsg as ovsg
        o = dict(data=hosts[q], x_axis=x, t_axis=t, veh_state_x=trk[q][0], veh_state_t=trk[q][1])
        ref = ovsg.virtual_shot_gather(o, pivot=p, start_x=p - 200.0, end_x=p + 200.0, wlen=2, **kw)[0]
        assert gio.gather_rel_err(got[u].double().cpu().numpy(), ref) < TOL, (u, q, j)
    del w, flat, got
    torch.cuda.empty_cache()


def test_sliding_merged_batches(device):
    """Two batches of trajectories over the same windows merged into ONE launch (UnitPlan.concat, the
    sliding bench's layout): every (class, pivot) stack equals the oracle's mean over both batches' units."""
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    from das_diff_veh_amd.synth import synth_batch_device
    from oracle import vsg as ovsg
    w, x, t, trk = _case(device, n=3, seed=14)
    _, _, _, trk2, _ = synth_batch_device(3, n_ch=300, n_t=8192, pivot=1100.0, seed=15, device=device,
                                          x_first=0.37, track_half=1500, chunk=1)
    kw = dict(include_other_side=True, norm=False)
    pch = np.arange(32, w.shape[1] - 32, 8)
    p1 = UnitPlan.sliding(x, t, trk, pch, 200.0, VsgParams(**kw))
    p2 = UnitPlan.sliding(x, t, trk2, pch, 200.0, VsgParams(**kw))
    plan = UnitPlan.concat([p1, p2])
    assert plan.n_pass == p1.n_pass + p2.n_pass
    assert np.array_equal(plan.pass_tab, np.concatenate([p1.pass_tab, p2.pass_tab]))
    slots = np.concatenate([p1.unit_pivot, p2.unit_pivot])  # one class: slot = pivot
    got = vsg.vsg_stack(vsg.flat_units(w, plan), plan, vsg.StackSchedule(slots, len(pch), chunk=8),
                        win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan)).double().cpu().numpy()
    host = w.double().cpu().numpy()
    refs = {}
    for pl, tr in ((p1, trk), (p2, trk2)):
        for u in range(pl.n_pass):
            refs.setdefault(int(pl.unit_pivot[u]), []).append(_oracle_unit(host, x, t, tr, pl, u, kw))
    for j, gs in refs.items():
        assert gio.gather_rel_err(got[j], ovsg.stack(gs)) < TOL, j
    assert len(refs) >= 2


def test_sliding_merged_validated(device):
    """The sliding bench's launch: two batches merged, windows validated in the stack launch through a
    UnitScan (window per (batch, pass), every unit taking its pass's validity).  Clean windows: the
    class stacks equal vsg_stack's; a NaN far from every gather in one window makes exactly the slots
    holding that window's units NaN (the reference's data / ||data||_F, apis/virtual_shot_gather.py:125)."""
    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    from das_diff_veh_amd.synth import synth_batch_device
    w, x, t, trk = _case(device, n=3, seed=14)
    _, _, _, trk2, _ = synth_batch_device(3, n_ch=300, n_t=8192, pivot=1100.0, seed=15, device=device,
                                          x_first=0.37, track_half=1500, chunk=1)
    prm = VsgParams(include_other_side=True, norm=False)
    pch = np.arange(32, w.shape[1] - 32, 8)
    p1 = UnitPlan.sliding(x, t, trk, pch, 200.0, prm)
    p2 = UnitPlan.sliding(x, t, trk2, pch, 200.0, prm)
    plan = UnitPlan.concat([p1, p2])
    n, C = w.shape[0], w.shape[1]
    scan = vsg.UnitScan(np.tile(np.arange(n) * C, 2), np.concatenate([p1.unit_window, p2.unit_window + n]), C)
    slots = np.concatenate([p1.unit_pivot, p2.unit_pivot])
    sched = vsg.StackSchedule(slots, len(pch), chunk=8)
    flat = vsg.flat_units(w, plan)
    ref = vsg.vsg_stack(flat, plan, sched, win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan)).double().cpu().numpy()
    sc = vsg.vsg_scales(flat, plan, validity=False)
    got = vsg.vsg_stack_validated(flat, plan, sched, scales=sc, scan=scan).double().cpu().numpy()
    used = np.unique(slots)
    assert np.all(np.isfinite(got[used]))
    assert max(gio.gather_rel_err(got[j], ref[j]) for j in used) < 1e-5
    w[1, C - 1, 7] = float("nan")  # the last channel's first samples: outside every gather's slices
    got = vsg.vsg_stack_validated(flat, plan, sched, scales=sc, scan=scan).double().cpu().numpy()
    bad = np.unique(slots[np.concatenate([p1.unit_window, p2.unit_window]) == 1])
    assert bad.size >= 1
    for j in used:
        if j in bad:
            assert np.all(np.isnan(got[j])), j
        else:
            assert gio.gather_rel_err(got[j], ref[j]) < 1e-5, j
