#!/usr/bin/env python
"""Throughput bench of the vehicle-pass imaging hot path on MI355X (one process per GPU).

Workload (default = BASELINE.json configs[1], "700_weights + 680_weights"): two synthetic window
sets, one per pivot (700 m and 680 m), each 1,895 vehicle passes of 60 channels x 5,500 samples
(8.16 m, dt = 0.004 s), split into heavy / mid / light classes of 103 / 1,058 / 734 passes
(imaging_diff_weight.ipynb#cell8).  One step = for every pivot: the per-pass amplitude scales,
the two-sided VSG of every pass fused with the per-class stack (sum / len), [multi-GPU: one
all-reduce of the partial class stacks], then the f-v image of every class stack
(compute_disp_image(end_x=0, start_x=-200): 1,000 velocities x 242 frequencies).
Inputs are resident in HBM before the timed region; the host-side index tables are built once.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload weights|speeds|synth10k|sliding]

synth10k (BASELINE.json configs[2]): 10,240 passes x 1,024 channels x 8,192 samples, single pivot
at channel 512, all channels in the gather aperture, speed-tercile classes.  The job (335 GB of
fp32 windows) exceeds HBM, so a pool of 512 passes is resident and a step images the 10,240 passes
as 20 batches over that pool, each batch with its own 512 per-pass trajectories (index tables);
window contents repeat across batches, the per-pass work does not.

sliding (BASELINE.json configs[3]): 4,096-channel x 8,192-sample windows imaged at sliding pivots
(every 8 channels, +-200 m) -- one unit per (pass, pivot crossed inside the window), slots = speed
class x pivot, one f-v image per slot (SlidingSet).  12,544 passes per GPU per step (100k over 8
GPUs), 49 batches over a resident pool of 256 windows (34 GB).

Prints ONE JSON line (rank 0).  `value` = vehicle-pass windows per second over all ranks.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from das_diff_veh_amd.disp import DispPlan, fk_grid, fv_from_fk  # noqa: E402
from das_diff_veh_amd.distributed import allreduce_stacks, max_over_ranks  # noqa: E402
from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry  # noqa: E402
from das_diff_veh_amd.synth import TRACK_DT, synth_batch_device  # noqa: E402
from das_diff_veh_amd.vsg import StackSchedule, vsg_scales, vsg_stack, window_sumsq  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 (non-packed) f32 VALU instruction every 4 cycles per SIMD
# (16 lanes), at the 2,400 MHz max clock (MI355X_MICROARCH.md).  = 78.6 TFLOP/s of non-packed f32 FMA.
VALU_PEAK_INSTR_S = 256 * 4 * 2.4e9 / 4

WORKLOADS = {
    # name: (list of (pivot, start_x, end_x, class counts), n_ch, n_t, description, options)
    "weights": ([(700.0, 500.0, 900.0, (103, 1058, 734)), (680.0, 480.0, 880.0, (103, 1058, 734))], 60, 5500,
                "configs[1]: 700_weights + 680_weights, heavy/mid/light 103/1058/734 per pivot, 60ch x 5500", {}),
    "speeds": ([(700.0, 500.0, 900.0, (330, 1442, 336))], 60, 5500,
               "configs[0]-shape: 700_speeds, fast/mid/slow 330/1442/336, 60ch x 5500", {}),
    "sliding": ([(None, None, None, 12544)], 4096, 8192,
                "configs[3]: synthetic passes x 4096ch x 8192, sliding pivots every 8 channels (+-200 m, 49 rows), "
                "each pass imaged at every pivot it crosses inside its window; 12,544 passes per GPU (100k over 8) "
                "as 49 batches over a resident pool of 256 passes; speed classes x pivots stacked, f-v image per "
                "(class, pivot)",
                dict(sliding=True, pool=256, pivot_every=8, half_aperture=200.0, gen_chunk=2)),
    "synth10k": ([(4178.0, 0.0, 8400.0, 10240)], 1024, 8192,
                 "configs[2]: synthetic 10,240 passes x 1024ch x 8192, pivot = channel 512, all channels, "
                 "speed-tercile classes; 20 batches over a resident pool of 512 passes",
                 dict(pool=512, x_first=0.37, track_half=4300, gen_chunk=8)),
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


class Batch:
    """One launch's worth of passes: their index tables and class schedule over the resident windows
    (``win`` / ``sumsq``: the launch view of the windows and its per-pass ||window||_F^2)."""

    def __init__(self, plan, sched, win=None, sumsq=None, scales=None):
        self.plan, self.sched = plan, sched
        self.win, self.sumsq, self.scales = win, sumsq, scales


class PivotSet:
    """One window set imaged at one pivot: device windows, index tables, class schedule.

    ``counts`` is either the per-class pass counts (all passes resident) or, with options["pool"],
    the total number of passes, imaged in batches of `pool` resident windows (speed-tercile classes)."""

    def __init__(self, pivot, start_x, end_x, counts, n_ch, n_t, seed, device, world, rank, opts, chunk=8):
        pool = opts.get("pool")
        n = pool or int(sum(counts))
        self.n = n
        t0 = time.time()
        self.windows, x_axis, t_axis, trk, _ = synth_batch_device(
            n, n_ch=n_ch, n_t=n_t, pivot=pivot, seed=seed, device=device, x_first=opts.get("x_first"),
            track_half=opts.get("track_half", 350), chunk=opts.get("gen_chunk", 64))
        self.t_gen = time.time() - t0
        t0 = time.time()
        self.prm = VsgParams(pivot=pivot, start_x=start_x, end_x=end_x, wlen=2, norm=False, include_other_side=True)
        rng = np.random.default_rng(seed + 7)
        if pool:
            n_total = int(counts)
            n_batch = -(-n_total // pool)
            xs_trk = trk[0][0]
            speeds = rng.uniform(15.0, 30.0, n_batch * pool)
            tcs = t_axis[n_t // 2] + rng.uniform(-1.0, 1.0, n_batch * pool)
            # speed terciles by rank (exact, equal-as-possible counts: every rank has the same class
            # sizes, so the global counts are world x the local ones)
            slots_all = np.empty(speeds.size, dtype=np.int64)
            slots_all[np.argsort(speeds, kind="stable")] = np.arange(speeds.size) * 3 // speeds.size
            counts = np.bincount(slots_all, minlength=3)
            trks = [(xs_trk, np.round((tc + (xs_trk - pivot) / v) / TRACK_DT) * TRACK_DT) for v, tc in zip(speeds, tcs)]
            batch_trk = [trks[b * pool:(b + 1) * pool] for b in range(n_batch)]
            batch_slots = [slots_all[b * pool:(b + 1) * pool] for b in range(n_batch)]
        else:
            batch_trk = [trk]
            batch_slots = [rng.permutation(np.repeat(np.arange(len(counts)), counts))]
        self.n_total = sum(len(t) for t in batch_trk)
        global_counts = np.asarray(counts) * world  # every rank holds its own full set (weak scaling)
        self.batches = []
        for bt, bs in zip(batch_trk, batch_slots):
            geoms = [pass_geometry(x_axis, t_axis, vx, vt, self.prm) for vx, vt in bt]
            plan = VsgPlan(geoms, self.prm, n_ch, n_t)
            self.batches.append(Batch(plan, StackSchedule(bs, len(counts), chunk=chunk, counts=global_counts)))
            self.batches[-1].slots = bs
        self.plan = self.batches[0].plan
        self.t_plan = time.time() - t0
        self.gx, self.gt = geoms[0].gather_x_axis, geoms[0].gather_t_axis
        self.stack = torch.zeros((len(counts), self.plan.R, self.plan.w), dtype=torch.float32, device=device)
        self.scales = torch.empty((n, 2), dtype=torch.float32, device=device)
        # ||window||_F^2 is a property of the resident windows (validity: finite, not all zero ->
        # the reference's data / ||data||_F), computed once at ingest like the index tables
        self.sumsq = window_sumsq(self.windows)
        s = int(np.abs(self.gx - (-200.0)).argmin())
        e = int(np.abs(self.gx - 0.0).argmin())
        self.disp_rows = (s, e + 1)
        self.disp = DispPlan(e + 1 - s, self.plan.w, 8.16, self.gt[1] - self.gt[0], np.arange(0.8, 25, 0.1),
                             np.arange(200, 1200))
        self.fv = torch.empty((len(counts), self.disp.nV, self.disp.nF), dtype=torch.float32, device=device)
        self.bytes_stack = [b.plan.algorithmic_bytes(out_rows=len(counts) * self.plan.R) for b in self.batches]
        self.host = (x_axis, t_axis, batch_trk[0])
        for b in self.batches:
            b.win, b.sumsq, b.scales = self.windows, self.sumsq, self.scales
        self.units = self.n_total


class SlidingSet:
    """BASELINE configs[3]: a pool of long-fiber windows imaged at sliding pivots (UnitPlan).

    Every batch gives the pool new per-pass trajectories (crossing point uniform along the fiber,
    15-30 m/s, crossing at mid-window); a pass becomes one unit per pivot it crosses inside its
    window (all rows with full-length slices on both sides).  Slots = speed class x pivot with
    fixed class edges (20, 25 m/s), so that every rank's slots mean the same thing; the class means
    use the GLOBAL unit count per slot (one all-reduce of the counts at setup)."""

    def __init__(self, n_total, n_ch, n_t, seed, device, world, rank, opts, chunk=8):
        from das_diff_veh_amd.plan import UnitPlan, sliding_pivots
        from das_diff_veh_amd.vsg import flat_units, unit_sumsq
        pool = opts["pool"]
        self.n = pool
        t0 = time.time()
        self.windows, x_axis, t_axis, _, _ = synth_batch_device(
            pool, n_ch=n_ch, n_t=n_t, pivot=n_ch * 8.16 / 2, seed=seed, device=device, x_first=0.37,
            track_half=10, chunk=opts.get("gen_chunk", 2))
        self.t_gen = time.time() - t0
        t0 = time.time()
        self.prm = VsgParams(wlen=2, norm=False, include_other_side=True)
        edge = 4 * opts["pivot_every"]
        pch = np.arange(edge, n_ch - edge, opts["pivot_every"])
        n_piv = pch.size
        rng = np.random.default_rng(seed + 7)
        n_batch = -(-int(n_total) // pool)
        self.n_total = n_batch * pool
        sumsq = window_sumsq(self.windows)
        plans, slot_l = [], []
        for _ in range(n_batch):
            x0 = rng.uniform(x_axis[edge], x_axis[-edge], pool)
            v = rng.uniform(15.0, 30.0, pool)
            tc = t_axis[n_t // 2] + rng.uniform(-1.0, 1.0, pool)
            trk = []
            for xa, va, ta in zip(x0, v, tc):
                xs = np.arange(np.floor(xa) - 800.0, np.floor(xa) + 801.0)
                trk.append((xs, np.round((ta + (xs - xa) / va) / TRACK_DT) * TRACK_DT))
            plan = UnitPlan.sliding(x_axis, t_axis, trk, pch, opts["half_aperture"], self.prm)
            cls = np.digitize(v[plan.unit_window], [20.0, 25.0])
            plans.append(plan)
            slot_l.append(cls * n_piv + plan.unit_pivot)
        n_slot = 3 * n_piv
        counts = np.bincount(np.concatenate(slot_l), minlength=n_slot)
        if world > 1:
            ct = torch.as_tensor(counts, dtype=torch.int64, device=device)
            dist.all_reduce(ct)
            counts = ct.cpu().numpy()
        self.batches = []
        for plan, sl in zip(plans, slot_l):
            b = Batch(plan, StackSchedule(sl, n_slot, chunk=chunk, counts=counts), win=flat_units(self.windows, plan),
                      sumsq=unit_sumsq(sumsq, plan),
                      scales=torch.empty((plan.n_pass, 2), dtype=torch.float32, device=device))
            self.batches.append(b)
        self.units = sum(p.n_pass for p in plans)
        self.plan = plans[0]
        self.t_plan = time.time() - t0
        R, w = self.plan.R, self.plan.w
        dt = t_axis[1] - t_axis[0]
        pv, st, en, _ = sliding_pivots(x_axis, pch[:1], opts["half_aperture"])
        self.gx = x_axis[st[0]:en[0]] - x_axis[pv[0]]
        self.gt = (np.arange(w) - w // 2) * dt
        self.stack = torch.zeros((n_slot, R, w), dtype=torch.float32, device=device)
        s = int(np.abs(self.gx - (-200.0)).argmin())
        e = int(np.abs(self.gx - 0.0).argmin())
        self.disp_rows = (s, e + 1)
        self.disp = DispPlan(e + 1 - s, w, 8.16, dt, np.arange(0.8, 25, 0.1), np.arange(200, 1200))
        self.fv = torch.empty((n_slot, self.disp.nV, self.disp.nF), dtype=torch.float32, device=device)
        self.bytes_stack = [p.algorithmic_bytes(out_rows=n_slot * R) for p in plans]
        self.host = None


def build(workload, device, world, rank, chunk=8):
    sets, n_ch, n_t, desc, opts = WORKLOADS[workload]
    out = []
    if opts.get("sliding"):
        return [SlidingSet(sets[0][3], n_ch, n_t, seed=1000 * rank + 3, device=device, world=world, rank=rank,
                           opts=opts, chunk=chunk)], desc
    for i, (pivot, sx, ex, counts) in enumerate(sets):
        out.append(PivotSet(pivot, sx, ex, counts, n_ch, n_t, seed=1000 * rank + 17 * i + 3, device=device,
                            world=world, rank=rank, opts=opts, chunk=chunk))
    return out, desc


def share_class_buffers(sets):
    """Put every pivot's class stacks (and f-v images) in ONE HBM buffer when the pivots share the
    gather geometry and the dispersion plan, so the step's f-v chain (tdft, FK contraction, f-v
    sampling) runs once over all class images instead of once per pivot: those launches are
    latency-bound at a few images each.  Returns (stack, fv, plan, rows) or None."""
    s0 = sets[0]
    if len(sets) < 2 or not all(hasattr(s, "disp_rows") for s in sets):
        return None
    p0 = s0.disp
    for s in sets[1:]:
        p = s.disp
        if (s.disp_rows != s0.disp_rows or s.stack.shape[1:] != s0.stack.shape[1:]
                or (p.nch, p.nt, p.dx, p.dt) != (p0.nch, p0.nt, p0.dx, p0.dt)
                or not np.array_equal(p.freqs, p0.freqs) or not np.array_equal(p.vels, p0.vels)):
            return None
    n = [s.stack.shape[0] for s in sets]
    stack = torch.zeros((sum(n),) + tuple(s0.stack.shape[1:]), dtype=s0.stack.dtype, device=s0.stack.device)
    fv = torch.empty((sum(n),) + tuple(s0.fv.shape[1:]), dtype=s0.fv.dtype, device=s0.fv.device)
    o = 0
    for s, k in zip(sets, n):
        s.stack, s.fv = stack[o:o + k], fv[o:o + k]
        o += k
    return stack, fv, p0, s0.disp_rows


def merge_pivot_sets(sets, shared, chunk=8):
    """One launch per step for every pivot's passes: the windows of all pivots in one resident
    buffer and one index table (each pass carries its own pivot row), class slots numbered across
    the pivots, so `vsg_scales` and `vsg_stack` run once over all passes instead of once per pivot
    and the stacks land in the shared class buffer.  Returns a set-like object, or None when the
    pivots do not share (rows, w, hop, flags) or are imaged in several batches."""
    from types import SimpleNamespace
    if shared is None or any(len(s.batches) != 1 or not hasattr(s.batches[0], "slots") for s in sets):
        return None
    if len({s.prm.flags for s in sets}) != 1:
        return None
    p0 = sets[0].batches[0].plan
    try:
        plan = VsgPlan([g for s in sets for g in s.batches[0].plan.geoms], sets[0].prm, p0.n_ch, p0.n_t)
    except ValueError:
        return None
    win = torch.cat([s.windows for s in sets])
    sumsq = torch.cat([s.sumsq for s in sets])
    slots, counts, off, o = [], [], 0, 0
    for s in sets:
        b = s.batches[0]
        slots.append(np.asarray(b.slots) + off)
        counts.append(np.asarray(b.sched.counts))
        off += b.sched.n_slot
        n = s.windows.shape[0]
        s.windows = b.win = win[o:o + n]  # the per-pivot views share the merged buffer
        s.sumsq = b.sumsq = sumsq[o:o + n]
        o += n
    sched = StackSchedule(np.concatenate(slots), off, chunk=chunk, counts=np.concatenate(counts))
    batch = Batch(plan, sched, win=win, sumsq=sumsq,
                  scales=torch.empty((plan.n_pass, 2), dtype=torch.float32, device=win.device))
    return SimpleNamespace(batches=[batch], stack=shared[0], fv=shared[1], disp=shared[2], disp_rows=shared[3],
                           plan=plan, bytes_stack=[plan.algorithmic_bytes(out_rows=off * plan.R)])


def launches(sets):
    return sum(len(s.batches) for s in sets)


def step(sets, world, ev=None, shared=None):
    k = 0
    for s in sets:
        for j, b in enumerate(s.batches):
            vsg_scales(b.win, b.plan, out=b.scales, win_sumsq=b.sumsq)
            if ev is not None:
                ev[k][0].record()
            vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=s.stack, accumulate=j > 0)
            if ev is not None:
                ev[k][1].record()
            k += 1
    if world > 1:
        allreduce_stacks([shared[0]] if shared is not None else [s.stack for s in sets])
    if shared is not None:  # every pivot's class images in one f-v chain
        stack, fv, plan, (a, b) = shared
        fv_from_fk(fk_grid(stack[:, a:b, :], plan), plan, out=fv)
        return
    for s in sets:
        a, b = s.disp_rows
        fv_from_fk(fk_grid(s.stack[:, a:b, :], s.disp), s.disp, out=s.fv)


def cpu_baseline(sets, budget_s=20.0, workers=None):
    """Reference-structured CPU path (oracle/ref_loop.py) on a bounded sample of the same windows.

    1 core: the bench windows themselves (host copies) for about budget_s / 2, plus one f-v image
    per set.  All cores: `workers` single-threaded processes (spawned, no GPU state; the box's CPU
    share is 16) each looping over a saved sample of the windows for budget_s / 2; the value is the
    aggregate windows/s, extrapolated with the 1-core image cost to one full step."""
    import multiprocessing as mp
    import tempfile

    from oracle import ref_loop
    torch.set_num_threads(1)
    workers = workers or max(1, min(16, os.cpu_count() or 1))
    n_win, t_win, t_img, n_img = 0, 0.0, 0.0, 0
    t_start = time.time()
    one_budget = budget_s / 2
    per_set = max(4, int(one_budget / 0.01 / max(len(sets), 1)))
    samples = []
    for s in sets:
        x_axis, t_axis, trk = s.host
        k = min(per_set, s.n, max(4, int(2e9 / (8 * s.windows[0].numel()))))  # host copy <= 2 GB
        host = s.windows[:k].to("cpu", torch.float64).numpy()
        samples.append((host[:16].astype(np.float32), x_axis, t_axis, trk[:16], s.prm))
        t0 = time.time()
        acc = None
        for i in range(k):
            g, gx, gt = ref_loop.gather(host[i], x_axis, t_axis, trk[i][0], trk[i][1], s.prm.pivot, s.prm.start_x,
                                        s.prm.end_x)
            acc = g if acc is None else acc + g
            if time.time() - t_start > one_budget:
                k = i + 1
                break
        t_win += time.time() - t0
        n_win += k
        t0 = time.time()
        ref_loop.disp_image(acc / k, gx, gt)
        t_img += time.time() - t0
        n_img += 1
    per_window = t_win / n_win
    per_image = t_img / n_img
    total_windows = sum(s.n_total for s in sets)
    total_images = sum(s.stack.shape[0] for s in sets)
    rate1 = total_windows / (per_window * total_windows + per_image * total_images)
    # all cores: single-threaded worker processes (plain python, no torch / GPU state) over a saved
    # sample of the first set's windows, all running at once
    import subprocess
    host, x_axis, t_axis, trk, prm = samples[0]
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "sample.npz")
        np.savez(path, wins=host, x_axis=x_axis, t_axis=t_axis, vx=np.stack([v for v, _ in trk]),
                 vt=np.stack([t for _, t in trk]), pivot=prm.pivot, start_x=prm.start_x, end_x=prm.end_x)
        procs = [subprocess.Popen([sys.executable, "-m", "oracle.ref_loop", path, str(w), str(budget_s / 2)],
                                  cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                 for w in range(workers)]
        res = []
        for pr in procs:
            try:
                out, _ = pr.communicate(timeout=budget_s * 4 + 60)
                done, secs = out.split()
                res.append((int(done), float(secs)))
            except Exception:  # a worker that failed or hung does not count
                pr.kill()
    if not res:
        raise RuntimeError("no CPU-baseline worker finished")
    workers = len(res)
    agg_window_rate = sum(n / t for n, t in res)
    step_s = total_windows / agg_window_rate + per_image * total_images / workers
    return dict(value=total_windows / step_s, unit="vehicle-pass windows/s", cores=workers, kind="port",
                sample=f"all cores: {workers} single-threaded processes x {budget_s / 2:.0f} s, {sum(n for n, _ in res)} "
                       f"windows (VSG two-sided), f-v images at the 1-core cost / {workers}; 1 core: {n_win} windows "
                       f"({per_window * 1e3:.1f} ms/window), {n_img} f-v images ({per_image * 1e3:.1f} ms/image) -> "
                       f"{rate1:.1f} windows/s; cpu={platform.processor() or platform.machine()}",
                value_1core=rate1)


def pmc_counter(kernel, workload, key):
    """Per-launch value of `key` for `kernel` from the newest committed PMC summary of this workload."""
    sfx = "" if workload == "weights" else "_" + workload
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_summary{sfx}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d and key in d[kernel]:
            return float(d[kernel][key]), os.path.basename(f)
    return None, None


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this
    workload (profiles/<round>_pmc_summary[_<workload>].json, written by tools/pmc.sh: FETCH_SIZE /
    WRITE_SIZE with the access-width calibration measured by tools/calib/fetch_calib).  (None, None)
    if absent."""
    sfx = "" if workload == "weights" else "_" + workload
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_summary{sfx}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d and "traffic_bytes" in d[kernel]:
            return float(d[kernel]["traffic_bytes"]), os.path.basename(f)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="weights", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--per-pivot-launch", action="store_true", help="one scales + stack launch per pivot")
    ap.add_argument("--per-pivot-fv", action="store_true", help="one f-v chain per pivot (no shared class buffer)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--chunk", type=int, default=8, help="passes per stack task (one wave, one gather row)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=device)

    sets, desc = build(args.workload, device, world, rank, chunk=args.chunk)
    torch.cuda.synchronize()
    log(f"[bench] rank {rank}: generated {sum(s.n for s in sets)} windows in {sum(s.t_gen for s in sets):.2f}s, "
        f"index tables in {sum(s.t_plan for s in sets):.2f}s; {sum(s.n_total for s in sets)} passes per step, "
        f"{launches(sets)} stack launches, R = {sets[0].plan.R}")

    shared = None if args.per_pivot_fv else share_class_buffers(sets)
    merged = None if args.per_pivot_launch else merge_pivot_sets(sets, shared, chunk=args.chunk)
    run = [merged] if merged is not None else sets  # what one step launches
    for _ in range(args.warmup):
        step(run, world, shared=shared)
    torch.cuda.synchronize()

    ev = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(launches(run))]
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(run, world, ev[k], shared=shared)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)

    stack_ms = np.array([[ev[k][i][0].elapsed_time(ev[k][i][1]) for i in range(launches(run))]
                         for k in range(args.steps)])
    windows_per_step = sum(s.n_total for s in sets) * world
    images_per_step = sum(s.stack.shape[0] for s in sets)
    # roofline of the dominant kernel (vsg_stack): algorithmic bytes per launch / mean launch time
    bytes_per_launch = float(np.mean([b for s in run for b in s.bytes_stack]))
    launch_s = float(stack_ms.mean()) / 1e3
    achieved = bytes_per_launch / launch_s / 1e9
    traffic, traffic_src = pmc_traffic("vsg_stackf_kernel", args.workload)
    res = {
        "metric": "vehicle-pass windows/sec -> stacked VSG + f-v images/sec; % HBM/MFMA roofline",
        "value": windows_per_step * args.steps / elapsed,
        "unit": "vehicle-pass windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated dispersive moving-source wavefield, per-pass trajectories)",
        "config": {"workload": args.workload, "description": desc, "windows_per_step_per_gpu": windows_per_step // world,
                   "class_images_per_step": images_per_step, "gather_rows": sets[0].plan.R, "w": sets[0].plan.w,
                   "parallelism": f"dp{world} (passes sharded, all-reduce of class stacks)", "chunk": args.chunk},
        "images_per_s": images_per_step * args.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "vsg_stackf_kernel", "bytes_per_launch": bytes_per_launch,
                     "launch_ms": launch_s * 1e3},
        "host_index_tables_s": sum(s.t_plan for s in sets),
    }
    # companion roofline: the stack kernel is VALU-issue bound (DESIGN.md "Roofline of the stack kernel"),
    # so report its VALU instructions per launch (PMC SQ_INSTS_VALU) / the live launch time vs the issue peak
    valu, valu_src = pmc_counter("vsg_stackf_kernel", args.workload, "SQ_INSTS_VALU")
    if valu is not None:
        res["valu_roofline"] = {"achieved": valu / launch_s, "peak": VALU_PEAK_INSTR_S, "unit": "wave-instr/s",
                                "frac": valu / launch_s / VALU_PEAK_INSTR_S, "instr_per_launch": valu,
                                "source": valu_src, "clock_assumed_ghz": 2.4,
                                "model": "every wave64 VALU instruction 4 cycles on its SIMD at the 2.4 GHz max clock; "
                                         "frac near or above 1 = VALU-issue bound (some instructions, e.g. moves "
                                         "and packed ops, issue in fewer cycles than the model charges)"}
    res["config"]["gather_units_per_step_per_gpu"] = sum(s.units for s in sets)
    res["config"]["stack_launches_per_step"] = launches(run)
    if any(s.host is None for s in sets):
        args.no_cpu_baseline = True  # the CPU loop images single-pivot windows (weights / speeds / synth10k)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(sets, args.cpu_budget)
        res["cpu_baseline"] = cb
        res["speedup_vs_cpu"] = res["value"] / cb["value"]
    else:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
