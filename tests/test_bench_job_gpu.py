"""bench.py's own step, at reduced pass counts, against the oracle (not only against itself).

The bench builds its jobs with device-derived tables (dvh_pass_geometry), per-batch validity, one
resident buffer for several pivots with per-pass channel axes (weights), and batches over a window
pool with their own trajectories (synth10k, BASELINE configs[2] geometry, R = 1023).  Here the same
build / step functions run on a few passes and the class stacks and f-v images are compared with
the float64 oracle (sum(images) / len(images), compute_disp_image).
"""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _oracle_classes(job, n_slot):
    from oracle import vsg as ovsg
    per_slot = [[] for _ in range(n_slot)]
    for cs_i, cs in enumerate(job.cpu_sets):
        host = cs["win"].double().cpu().numpy()
        for i, (vx, vt) in enumerate(cs["trk"][:host.shape[0]]):
            o = dict(data=host[i], x_axis=cs["x_axis"], t_axis=cs["t_axis"], veh_state_x=vx, veh_state_t=vt)
            p = cs["prm"]
            with np.errstate(all="ignore"):
                g = ovsg.virtual_shot_gather(o, include_other_side=True, norm=False, pivot=p.pivot, start_x=p.start_x,
                                             end_x=p.end_x, wlen=p.wlen)[0]
            per_slot[cs["slots"][i]].append(g)
    return [ovsg.stack(g) if g else None for g in per_slot]


def _check(job, refs, gx, gt):
    from oracle import disp as odisp
    got = job.stack.double().cpu().numpy()
    fv = job.fv.cpu().numpy()
    for s, ref in enumerate(refs):
        if ref is None:
            continue
        assert gio.gather_rel_err(got[s], ref) < TOL, s
        fref = odisp.compute_disp_image(ref, gx, gt, start_x=-200, end_x=0)
        assert np.abs(fv[s] - fref).max() / np.abs(fref).max() < TOL, s


def test_weights_job(device):
    import bench
    wl = dict(bench.WORKLOADS["weights"], pivots=[(700.0, 500.0, 900.0, (3, 4, 2)), (680.0, 480.0, 880.0, (2, 3, 2))])
    job = bench.build_resident(wl, device, 1, 0, "weak", chunk=2)
    bench.step(job, 1)
    bench.step(job, 1)  # a second step recomputes (tables, validity, stacks) from scratch
    sl = job.batches[0].slots
    o = 0
    for cs in job.cpu_sets:
        k = cs["win"].shape[0]
        cs["slots"] = sl[o:o + k]
        o += k
    refs = _oracle_classes(job, 6)
    cs = job.cpu_sets[0]
    p = cs["prm"]
    st, pv = int(np.argmax(cs["x_axis"] >= p.start_x)), int(np.argmax(cs["x_axis"] >= p.pivot))
    R = job.stack.shape[1]
    dt = cs["t_axis"][1] - cs["t_axis"][0]
    _check(job, refs, cs["x_axis"][st:st + R] - cs["x_axis"][pv], (np.arange(500) - 250) * dt)


def test_synth10k_job(device):
    import bench
    wl = dict(bench.WORKLOADS["synth10k"], n_total=6, pool=4, gen_chunk=2)
    job = bench.build_pool(wl, device, 1, 0, "weak", chunk=2)
    # 6 passes over a nominal pool of 4: two equal batches of 3 (no remainder launch)
    assert len(job.batches) == 2 and job.batches[0].plan.R == 1023
    assert [b.plan.n_pass for b in job.batches] == [3, 3] and job.windows.shape[0] == 3
    bench.step(job, 1)
    # pass i of the job lives in pool slot i % 3 during its batch
    cs = job.cpu_sets[0]
    slots = np.concatenate([b.slots for b in job.batches])
    wins = job.windows.double().cpu().numpy()
    from oracle import vsg as ovsg
    per_slot = [[] for _ in range(3)]
    p = cs["prm"]
    for i, (vx, vt) in enumerate(cs["trk"][:6]):
        o = dict(data=wins[i % 3], x_axis=cs["x_axis"], t_axis=cs["t_axis"], veh_state_x=vx, veh_state_t=vt)
        per_slot[slots[i]].append(ovsg.virtual_shot_gather(o, include_other_side=True, norm=False, pivot=p.pivot,
                                                           start_x=p.start_x, end_x=p.end_x, wlen=p.wlen)[0])
    refs = [ovsg.stack(g) if g else None for g in per_slot]
    x = cs["x_axis"]
    dt = cs["t_axis"][1] - cs["t_axis"][0]
    _check(job, refs, x[0:1023] - x[512], (np.arange(500) - 250) * dt)


def test_synth10k_full_job_properties(device):
    """The bench's synth10k job at its FULL size (BASELINE configs[2]: 10 240 passes of 1 024 x 8 192 as
    5 batches of 2 048 over the window pool), through size-independent properties:
      * the validated launch (correlation + class stack + validity of every window sample in one launch)
        equals the separate path (dvh_window_sumsq launch, then the plain stack launch) to 1e-5;
      * stacking is linear: the step's class stacks equal the count-weighted sum of the batches'
        own class means;
      * every class image is finite and a step is reproducible to fp32 atomic-order rounding."""
    import torch

    import bench
    job = bench.build("synth10k", device, 1, 0)
    assert len(job.batches) == 5 and sum(b.plan.n_pass for b in job.batches) == 10240
    bench.step(job, 1, fused=True)
    fused, fv = job.stack.clone(), job.fv.clone()
    bench.step(job, 1, fused=False)
    sep = job.stack.clone()
    scale = float(sep.abs().max())
    assert float((fused - sep).abs().max()) <= 1e-5 * scale
    assert torch.isfinite(fv).all() and torch.isfinite(fused).all()
    # linearity: per-batch class means (batch-local counts), weighted by the batch's share of each class
    from das_diff_veh_amd.vsg import StackSchedule, vsg_scales, vsg_stack_validated
    total = torch.zeros_like(fused)
    counts = np.bincount(np.concatenate([b.slots for b in job.batches]), minlength=3)
    for b in job.batches:
        b.plan.derive()
        sc = vsg_scales(b.win, b.plan, validity=False)
        local = np.bincount(b.slots, minlength=3)
        part = vsg_stack_validated(b.win, b.plan, StackSchedule(b.slots, 3, chunk=8), scales=sc)
        total += part * torch.as_tensor(local / counts, dtype=torch.float32, device=device)[:, None, None]
    assert float((total - fused).abs().max()) <= 1e-5 * scale
    bench.step(job, 1, fused=True)
    assert float((job.stack - fused).abs().max()) <= 1e-5 * scale


def test_synth10k_w499_full_job_properties(device):
    """The bench's synth10k job at w = 499 (`bench.py --w499`: dt = 0.004000000000001336, the zero-padded
    1 024-point engine) at FULL size: the validated launch equals the separate path (window_sumsq, then the
    plain padded stack kernel) to 1e-5, every class image is finite and a step is reproducible."""
    import bench
    from das_diff_veh_amd.synth import DT_W499
    wl = dict(bench.WORKLOADS["synth10k"], t0=DT_W499)
    job = bench.build_pool(wl, device, 1, 0, "weak", chunk=8)
    assert job.batches[0].plan.w == 499 and sum(b.plan.n_pass for b in job.batches) == 10240
    bench.step(job, 1, fused=True)
    fused, fv = job.stack.clone(), job.fv.clone()
    bench.step(job, 1, fused=False)
    sep = job.stack.clone()
    scale = float(sep.abs().max())
    assert scale > 0 and float((fused - sep).abs().max()) <= 1e-5 * scale
    assert bool(fv.isfinite().all()) and bool(fused.isfinite().all())
    bench.step(job, 1, fused=True)
    assert float((job.stack - fused).abs().max()) <= 1e-5 * scale


def test_sliding_job(device):
    """bench.build_sliding as built (configs[3]'s job at a reduced size): per-batch trajectories over a resident
    pool, (class, pivot) slots with the fixed 20 / 25 m/s class edges, batches merged into one UnitPlan.concat
    launch, every window validated through the UnitScan tiling.  Every used slot's stack equals the oracle's
    mean over that slot's units -- each unit imaged at its own pivot +- 200 m on its pool window with its own
    batch's trajectory (apis/virtual_shot_gather.py:165-192) -- and its f-v image equals the oracle's."""
    import bench
    from oracle import disp as odisp
    from oracle import vsg as ovsg
    wl = dict(bench.WORKLOADS["sliding"], n_total=6, pool=3, n_ch=600, merge=2, gen_chunk=3)
    job = bench.build_sliding(wl, device, 1, 0, "weak", chunk=2)
    assert len(job.batches) == 1 and job.batches[0].n_merged == 2  # 2 batches of 3 passes, one merged launch
    bench.step(job, 1)
    cu = job.cpu_units
    x_axis, t_axis, pch, half = cu["x_axis"], cu["t_axis"], cu["pch"], cu["half"]
    wins = job.windows.double().cpu().numpy()
    n_slot = job.stack.shape[0]
    per_slot = [[] for _ in range(n_slot)]
    axes = {}
    for b in job.batches:
        u0 = 0
        for k in range(b.n_merged):
            plan, trk = job.plans[b.first_batch + k], job.trks[b.first_batch + k]
            for u in range(plan.n_pass):
                q, j = int(plan.unit_window[u]), int(plan.unit_pivot[u])
                p = float(x_axis[pch[j]])
                o = dict(data=wins[q], x_axis=x_axis, t_axis=t_axis, veh_state_x=trk[q][0], veh_state_t=trk[q][1])
                g, gx, gt = ovsg.virtual_shot_gather(o, include_other_side=True, norm=False, pivot=p,
                                                     start_x=p - half, end_x=p + half, wlen=2)
                per_slot[int(b.slots[u0 + u])].append(g)
                axes[int(b.slots[u0 + u])] = (gx, gt)
            u0 += plan.n_pass
        assert u0 == b.plan.n_pass
    used = [s for s in range(n_slot) if per_slot[s]]
    assert len(used) >= 4
    got = job.stack.double().cpu().numpy()
    fv = job.fv.cpu().numpy()
    for s in range(n_slot):
        if not per_slot[s]:
            assert not np.any(got[s]), s  # an empty slot stays zero
            continue
        ref = ovsg.stack(per_slot[s])
        assert gio.gather_rel_err(got[s], ref) < TOL, s
        fref = odisp.compute_disp_image(ref, *axes[s], start_x=-200, end_x=0)
        assert np.abs(fv[s] - fref).max() / np.abs(fref).max() < TOL, s
