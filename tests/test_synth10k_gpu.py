"""GPU parity at the BASELINE configs[2] geometry (the bench's synth10k workload) against the oracle.

1024 channels x 8192 samples, dx 8.16 m, pivot = channel 512, start_x = 0 / end_x = 8400 (all channels,
R = 1023), dt = 0.0039999999999995595 (w = 500), two-sided, norm=False (VirtualShotGathersFromWindows'
setting).  Tables come from the device (dvh_pass_geometry), as in the bench step.  Four regular passes
(a slow, a fast and two bench-style ones): most rows' trajectory times fall outside the window, where
the reference reads [0, nsamp) (argmax of an all-False mask).  Two edge passes whose
shared pivot slice on one side is empty or shorter than a sub-window: that side's pivot row is 0, so
the reference's rows are x / 0 = +-inf (NaN where x == 0).  A window with a NaN in a channel that is
not a gather row makes its whole gather NaN (data / ||data||_F, apis/virtual_shot_gather.py:125).
"""
import numpy as np
import pytest

from tests import golden_io as gio
from tests.test_plan_gpu import synth10k_trajectories

pytestmark = pytest.mark.gpu
TOL = 1e-4
N, N_REG = 6, 4


@pytest.fixture(scope="module")
def batch(device):
    import torch

    from das_diff_veh_amd.plan import DevicePlan, VsgParams, pack_trajectories
    from das_diff_veh_amd.synth import synth_batch_device
    from das_diff_veh_amd.vsg import window_sumsq
    win, x_axis, t_axis, _, _ = synth_batch_device(N, n_ch=1024, n_t=8192, pivot=4178.0, seed=21, device=device,
                                                   x_first=0.37, track_half=10, chunk=2)
    trks = synth10k_trajectories(x_axis, t_axis, 5, N)
    prm = VsgParams(pivot=4178.0, start_x=0.0, end_x=8400.0, wlen=2, norm=False, include_other_side=True)
    plan = DevicePlan(x_axis, t_axis, *pack_trajectories(trks, device), prm, 1024).check()
    assert plan.R == 1023 and plan.w == 500
    win_nan = win.clone()
    win_nan[1, 1023, 8000] = float("nan")  # channel 1023 is outside the gather rows 0..1022
    torch.cuda.synchronize()
    return dict(win=win, win_nan=win_nan, x_axis=x_axis, t_axis=t_axis, trks=trks, prm=prm, plan=plan,
                sumsq=window_sumsq(win), sumsq_nan=window_sumsq(win_nan))


def _oracle(batch, i, nan=False, side=None):
    """The reference gather of pass i; side = 'f' / 'o': that side alone without the amax scale."""
    from oracle import vsg as ovsg
    data = (batch["win_nan"] if nan else batch["win"])[i].double().cpu().numpy()
    vx, vt = batch["trks"][i]
    o = dict(data=data, x_axis=batch["x_axis"], t_axis=batch["t_axis"], veh_state_x=vx, veh_state_t=vt)
    p = batch["prm"]
    kw = dict(norm=False, pivot=p.pivot, start_x=p.start_x, end_x=p.end_x, wlen=p.wlen)
    with np.errstate(all="ignore"):
        if side is not None:
            return ovsg.shot_gather(o, other_side=side == "o", norm_amp=False, **kw)[0]
        return ovsg.virtual_shot_gather(o, include_other_side=True, **kw)[0]


@pytest.fixture(scope="module")
def refs(batch):
    return [_oracle(batch, i) for i in range(N)]


@pytest.fixture(scope="module")
def gathers(batch):
    from das_diff_veh_amd.vsg import vsg_gathers, vsg_scales
    plan = batch["plan"]
    sc = vsg_scales(batch["win"], plan, win_sumsq=batch["sumsq"])
    return vsg_gathers(batch["win"], plan, sc).double().cpu().numpy()


def test_per_pass_gathers(gathers, refs):
    for i in range(N_REG):
        assert np.isfinite(refs[i]).all()
        assert gio.gather_rel_err(gathers[i], refs[i]) < TOL, i


def test_edge_passes_inf_rows(batch, gathers, refs):
    """Rows divided by a zero pivot-row amax: finite entries to 1e-4, NaN where the reference's are,
    +-inf where the reference's are, with the sign of the raw correlation wherever it is not at
    rounding level (|raw| > 1e-3 max |raw| of its side; fp32 and float64 disagree on the sign of
    values that are zero up to rounding)."""
    n_inf = 0
    for i in range(N_REG, N):
        ref, got = refs[i], gathers[i]
        if np.isfinite(ref).all():
            assert gio.gather_rel_err(got, ref) < TOL, i
            continue
        n_inf += 1
        assert np.array_equal(np.isnan(got), np.isnan(ref)), i
        assert np.array_equal(np.isinf(got), np.isinf(ref)), i
        fin = np.isfinite(ref)
        if fin.any():
            assert np.abs(got[fin] - ref[fin]).max() <= TOL * np.abs(ref[fin]).max(), i
        # which side is divided by zero: the one whose unscaled pivot row is all zero
        raw_f, raw_o = (_oracle(batch, i, side=s) for s in "fo")  # as laid out in the gather (flip included)
        raw = raw_o if not np.any(raw_o[512]) else raw_f
        inf = np.isinf(ref)
        big = np.abs(raw) > 1e-3 * np.abs(raw).max()
        chk = inf & big
        assert chk.sum() > 0.5 * inf.sum(), i
        assert np.array_equal(np.sign(got[chk]), np.sign(ref[chk])), i
    assert n_inf >= 1  # the late pass (the early one's other side is all 0 / 0 = NaN: not averaged)


def test_class_stack(batch, refs):
    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack
    from oracle import vsg as ovsg
    slots = np.array([0, 1, 0, 1, 2, 2])
    got = vsg_stack(batch["win"], batch["plan"], StackSchedule(slots, 3, chunk=2),
                    win_sumsq=batch["sumsq"]).double().cpu().numpy()
    for s in range(2):
        ref = ovsg.stack([refs[i] for i in np.where(slots == s)[0]])
        assert gio.gather_rel_err(got[s], ref) < TOL, s


def test_invalid_window_outside_rows(batch, refs):
    from das_diff_veh_amd.vsg import StackSchedule, vsg_gathers, vsg_scales, vsg_stack
    from oracle import vsg as ovsg
    plan = batch["plan"]
    ref_nan = _oracle(batch, 1, nan=True)
    assert np.isnan(ref_nan).all()
    g = vsg_gathers(batch["win_nan"], plan, vsg_scales(batch["win_nan"], plan, win_sumsq=batch["sumsq_nan"]))
    assert np.isnan(g[1].double().cpu().numpy()).all()
    slots = np.array([0, 1, 0, 1, 2, 2])
    got = vsg_stack(batch["win_nan"], plan, StackSchedule(slots, 3, chunk=4),
                    win_sumsq=batch["sumsq_nan"]).double().cpu().numpy()
    assert np.isnan(got[1]).all()
    assert gio.gather_rel_err(got[0], ovsg.stack([refs[0], refs[2]])) < TOL


def test_validated_stack(batch, refs):
    """The stack launch that also decides every window's validity (vsg_stack_validated) equals the
    oracle, and a NaN in a channel no gather row reads turns exactly its class NaN."""
    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack_validated
    from oracle import vsg as ovsg
    slots = np.array([0, 1, 0, 1, 2, 2])
    for key, bad in (("win", None), ("win_nan", 1)):
        got = vsg_stack_validated(batch[key], batch["plan"], StackSchedule(slots, 3, chunk=2)).double().cpu().numpy()
        for s in range(2):
            if s == bad:
                assert np.isnan(got[s]).all()
            else:
                ref = ovsg.stack([refs[i] for i in np.where(slots == s)[0]])
                assert gio.gather_rel_err(got[s], ref) < TOL, (key, s)


def test_validated_stack_receiver_slices(batch, refs):
    """Window validity inside the slices the correlation waves load (which the launch's scan may leave to
    them) and in the samples between them: a NaN in a gather row's receiver slice, an inf just past the end
    of another row's slice and an all-zero window each turn exactly their class NaN."""
    import torch

    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack_validated
    from oracle import vsg as ovsg
    plan = batch["plan"]
    seg = plan.host_seg_tab().reshape(plan.n_pass, plan.R, 2, 2)  # (start, len) per pass, row, side
    win = batch["win"]
    slots = np.array([0, 1, 0, 1, 2, 2])
    cases = []
    w = win.clone()  # pass 2 (slot 0): NaN inside row 100's forward receiver slice
    a, n = int(seg[2, 100, 0, 0]), int(seg[2, 100, 0, 1])
    assert n >= 500
    w[2, 100, a + 10] = float("nan")
    cases.append((w, {0}))
    w = win.clone()  # pass 3 (slot 1): -inf one sample past the end of row 700's other-side slice
    a, n = int(seg[3, 700, 1, 0]), int(seg[3, 700, 1, 1])
    assert n >= 500 and a + n < win.shape[2]
    w[3, 700, a + n] = float("-inf")
    cases.append((w, {1}))
    w = win.clone()  # pass 4 (slot 2): all zero (0 / 0 in the reference)
    w[4] = 0.0
    cases.append((w, {2}))
    for w, bad in cases:
        torch.cuda.synchronize()
        got = vsg_stack_validated(w, batch["plan"], StackSchedule(slots, 3, chunk=2)).double().cpu().numpy()
        for s in range(3):
            if s in bad:
                assert np.isnan(got[s]).all(), (bad, s)
            elif s < 2:
                ref = ovsg.stack([refs[i] for i in np.where(slots == s)[0]])
                assert gio.gather_rel_err(got[s], ref) < TOL, (bad, s)
            else:
                assert not np.isnan(got[s]).all(), (bad, s)


def test_stack_mixed_chunks(batch, refs):
    """Row tasks whose passes differ -- a regular pass with an edge pass (one side's pivot slice empty, so
    that side is 0 / 0 and not averaged) in one chunk -- take the per-pass path where the cross-pass packing
    (EngF500::direct_task) does not apply and the packed path where it does; both class means equal the
    oracle's.  (The other edge pass, whose rows are x / 0, is parked in a third slot.)"""
    from das_diff_veh_amd.vsg import StackSchedule, vsg_stack
    from oracle import vsg as ovsg
    fin = [i for i in range(N_REG, N) if np.isfinite(refs[i]).all()]
    assert fin
    e = fin[0]
    slots = np.array([0, 1, 1, 1, 2, 2])
    slots[e] = 0
    with np.errstate(all="ignore"):
        ref1 = ovsg.stack([refs[i] for i in (1, 2, 3)])
        ref0 = ovsg.stack([refs[i] for i in (0, e)])
    for chunk in (3, 2):
        got = vsg_stack(batch["win"], batch["plan"], StackSchedule(slots, 3, chunk=chunk),
                        win_sumsq=batch["sumsq"]).double().cpu().numpy()
        assert gio.gather_rel_err(got[1], ref1) < TOL, chunk
        assert gio.gather_rel_err(got[0], ref0) < TOL, chunk
