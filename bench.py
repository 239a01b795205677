#!/usr/bin/env python
"""Throughput bench of the vehicle-pass imaging hot path on MI355X (one process per GPU).

Default workload = BASELINE.json configs[2], "synth10k", the largest single-GPU configuration:
10,240 synthetic vehicle passes of 1,024 channels x 8,192 samples (8.16 m, dt = 0.004 s), one pivot
(channel 512), every channel a gather row (R = 1,023), speed-tercile classes.  The job's 335 GB of
fp32 windows exceed HBM, so a pool of 2,048 windows (69 GB) is resident and one step images the 10,240
passes as 5 batches over that pool, each batch with its own 2,048 trajectories (window contents repeat
across batches, the per-pass work does not).

One step, per batch, all on the device and on one stream:
  1. the batch's index tables from its trajectories      dvh_pass_geometry   (preprocessing_window)
  2. the windows' validity ||window||_F^2                 dvh_window_sumsq    (data / ||data||_F)
  3. the per-pass amplitude scales                        dvh_vsg_scales      (post_processing_XCF)
  4. the two-sided VSG of every pass fused with the class stack     dvh_vsg_stack
then [N > 1: one all-reduce of the partial class stacks] and the f-v image of every class stack
(compute_disp_image(end_x=0, start_x=-200): 1,000 velocities x 242 frequencies).  Only the windows
and the trajectories are resident before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload synth10k|weights|speeds|sliding|timelapse]
                    [--scaling weak|strong|both]

weak (default at N = 1): every rank images its own full job (value = N x the job per step).  strong:
ONE job of the configured size is split over the ranks (das_diff_veh_amd.distributed.shard_passes:
every class dealt round robin), class means with the global counts, one all-reduce.  both (default at
N > 1): the weak line, with the strong measurement of the same workload in its "strong_scaling" field.
weights (configs[1]): two pivots (700 m, 680 m) x 1,895 passes (heavy/mid/light 103/1,058/734) of
60 x 5,500 in ONE resident buffer, one launch of each kernel per step, 6 class images.
sliding (configs[3]): 4,096-channel windows imaged at every pivot they cross (host O(C + J) unit
tables); every pass's whole window validated inside the stack launch (134 MB per pass), see DESIGN.md.
timelapse (configs[4]): batched f-v images of daily stacks (512 gathers x 512 velocities x 1,000
frequencies per step and rank, no exchange: days shard over the ranks), value = f-v images/s.

Prints ONE JSON line (rank 0).  `value` = vehicle-pass windows per second over all ranks.

Multi-GPU: `python bench.py --gpus N` (N > 1) run without a launcher (no WORLD_SIZE in the environment)
starts the N ranks itself, one process per GPU, before anything here imports torch or touches HIP
(launch_ranks); under `torch.distributed.run --nproc-per-node N` every rank checks that the world
size equals --gpus.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="synth10k",
                    choices=("synth10k", "weights", "speeds", "sliding", "timelapse", "bootstrap", "prep",
                             "speeds-host"))
    ap.add_argument("--scaling", default=None, choices=("weak", "strong", "both"),
                    help="weak: every rank its own job; strong: one job split over the ranks; both (default for "
                         "N > 1): the weak line with the strong (fixed-job) measurement beside it")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--chunk", type=int, default=8, help="passes per stack task (one wave, one gather row)")
    ap.add_argument("--pool", type=int, default=None, help="resident windows (= passes per stack launch) of the pool "
                    "workloads (default: the workload's)")
    ap.add_argument("--sliding-merge", type=int, default=None,
                    help="sliding: batches of trajectories per stack launch (default: all 49 in one launch)")
    ap.add_argument("--separate-validity", action="store_true",
                    help="window_sumsq launch per batch instead of the validity scan inside the stack launch")
    ap.add_argument("--layout-out", default=None, help="write the launch layout (JSON) for tools/pmc_summary.py")
    ap.add_argument("--w499", action="store_true",
                    help="synth10k / weights / speeds on time axes whose dt = 0.004000000000001336 (w = int(wlen / dt) = "
                         "499, the reference's other operating point: zero-padded 1 024-point transforms)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="test hook: the ranks launch_ranks starts print their rank environment instead of benching")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n, poll_s=0.2, grace_s=10.0):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1), relay rank 0's output and
    return 0 when every rank exits 0.  Runs before torch is imported: this process never initialises HIP,
    and it starts children instead of replacing itself (no exec after a GPU was touched).

    All ranks are polled: the first rank that exits non-zero ends the run -- the others (blocked in a
    rendezvous or a collective waiting for it) are terminated, then killed after `grace_s` -- and its exit
    code and stderr tail are printed, so a failing rank never leaves the launch waiting for the
    process-group timeout."""
    import tempfile
    import time as _time
    port = str(_free_port())
    tmp = tempfile.mkdtemp(prefix="dvh_ranks_")
    procs, errs = [], []
    out0 = open(os.path.join(tmp, "rank0.out"), "w+")
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # rank 0's stderr streams through (progress lines); the other ranks' go to files, tailed on failure
        err = None if r == 0 else open(os.path.join(tmp, f"rank{r}.err"), "w+")
        errs.append(err)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL, stderr=err))
    failed = None
    while failed is None and any(p.returncode is None for p in procs):
        for r, p in enumerate(procs):
            if p.returncode is None and p.poll() is not None and p.returncode != 0:
                failed = r
                break
        else:
            _time.sleep(poll_s)
    if failed is not None:
        for p in procs:
            if p.returncode is None:
                p.terminate()
        t_end = _time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - _time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out0.seek(0)
    for line in out0.read().splitlines(True):  # the JSON line on stdout, anything else rank 0 printed on stderr
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
    sys.stdout.flush()
    rcs = [p.returncode for p in procs]
    rc = 0
    if failed is not None:
        rc = procs[failed].returncode
        tail = ""
        if errs[failed] is not None:
            errs[failed].seek(0)
            tail = "".join(errs[failed].read().splitlines(True)[-20:])
        print(f"[bench] rank {failed} exited with {rc}; the other ranks were stopped (exit codes {rcs})\n{tail}",
              file=sys.stderr, flush=True)
        rc = rc if rc > 0 else 1
    for f in [out0] + [e for e in errs if e is not None]:
        f.close()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    return rc


if __name__ == "__main__":
    _ARGS = parse_args()
    if "WORLD_SIZE" not in os.environ and _ARGS.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], _ARGS.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != _ARGS.gpus:
        print(f"[bench] --gpus {_ARGS.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: one rank per GPU expected",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if _ARGS.launch_dry_run:
        # test hook (tests/test_bench_launch.py): DVH_DRY_FAIL="rank:code" makes that rank exit with the code
        # while every other rank blocks, as ranks waiting in a collective for a dead peer do
        fail = os.environ.get("DVH_DRY_FAIL")
        if fail:
            fr, fc = (int(v) for v in fail.split(":"))
            if int(os.environ["RANK"]) == fr:
                print(f"[dry-run] rank {fr} fails with {fc}", file=sys.stderr, flush=True)
                sys.exit(fc)
            time.sleep(600)
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                             "MASTER_PORT")}), flush=True)
        sys.exit(0)

import numpy as np  # noqa: E402  (after the rank launch: the launching process never imports torch)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, ROOT)

from das_diff_veh_amd.disp import DispPlan, fk_grid, fv_from_fk  # noqa: E402
from das_diff_veh_amd.distributed import allreduce_stacks, max_over_ranks, shard_passes  # noqa: E402
from das_diff_veh_amd.plan import DevicePlan, VsgParams  # noqa: E402
from das_diff_veh_amd.synth import DT_W499, DT_W500, TRACK_DT, synth_batch_device  # noqa: E402
from das_diff_veh_amd.vsg import StackSchedule, vsg_scales, vsg_stack, vsg_stack_validated, window_sumsq  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMD-32s, one wave64 VALU instruction per 2 cycles per SIMD once >= 2
# waves share the SIMD (MI355X_MICROARCH.md "Wave scheduling" and the v_fma_f32 row of the cycle
# constants), at the 2,400 MHz max clock = 1.229 T wave-instructions/s.
VALU_PEAK_INSTR_S = 256 * 4 * 2.4e9 / 2

WORKLOADS = {
    "synth10k": dict(kind="pool", config="configs[2]", pivot=(4178.0, 0.0, 8400.0), n_total=10240, n_ch=1024, n_t=8192,
                     pool=2048, x_first=0.37, gen_chunk=8, track_half=4300,
                     desc="configs[2]: synthetic 10,240 passes x 1024 ch x 8192, pivot = channel 512, all channels "
                          "(R = 1023), speed-tercile classes; 5 batches of 2048 over a resident window pool (69 GB), each "
                          "batch with its own trajectories"),
    "weights": dict(kind="resident", config="configs[1]",
                    pivots=[(700.0, 500.0, 900.0, (103, 1058, 734)), (680.0, 480.0, 880.0, (103, 1058, 734))],
                    n_ch=60, n_t=5500, gen_chunk=64, track_half=350,
                    desc="configs[1]: 700_weights + 680_weights, heavy/mid/light 103/1058/734 per pivot, 60 ch x 5500, "
                         "both pivots in one launch"),
    "speeds": dict(kind="resident", config="configs[0]-shape", pivots=[(700.0, 500.0, 900.0, (330, 1442, 336))],
                   n_ch=60, n_t=5500, gen_chunk=64, track_half=350,
                   desc="configs[0]-shape: 700_speeds, fast/mid/slow 330/1442/336, 60 ch x 5500"),
    "timelapse": dict(kind="timelapse", config="configs[4]", B=512, nch=25, nt=500, nV=512, nF=1000,
                      desc="configs[4]: time-lapse daily stacks, the f-v image (512 velocities x 1,000 frequencies, "
                           "1-25 Hz, 200-1200 m/s) of 512 gathers of 25 ch x 500 lags per step and rank (a day's "
                           "stacks at 512 pivots): time DFT + channel contraction on the fp64 MFMA pipe, FITPACK "
                           "bilinear + Savitzky-Golay (fp64 MFMA); every rank images its own days"),
    "speeds-host": dict(kind="host", config="configs[0]-shape, host-fed", classes=(330, 1442, 336), n_ch=60, n_t=5500,
                        desc="configs[0]-shape through the drop-in API as a notebook calls it: "
                             "VirtualShotGathersFromWindows(windows_<class>).get_images(include_other_side=True, pivot=700, "
                             "start_x=500, end_x=900, wlen=2) for fast / mid / slow (330 / 1,442 / 336 NumPy float32 "
                             "windows of 60 x 5,500 in host memory), each class's avg_image back on the host"),
    "bootstrap": dict(kind="bootstrap", config="SURVEY §8(f) row 1", n=1442, max_size=60, bt_times=30,
                      desc="the notebooks' convergence_test (imaging_diff_speed.ipynb#cell30-31) for one class: 1,442 "
                           "passes of 60 x 5,500 (pivot 700 m, 500-900 m), bt_size 1..60 x 30 resamples, 4 ridge modes "
                           "(#cell25 sigma / ref_freq_idx / bands / reference curves); gathers from the resident "
                           "windows, resample stacks, f-v images (242 x 1,000) and ridges every step"),
    "prep": dict(kind="prep", config="SURVEY §8(f) row 2", n_ch=1024, seconds=60.0, dt=0.004,
                 desc="TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71) of a "
                      "continuous float32 record of 1,024 channels x 60 s at 250 Hz: bandpass_data (order-10 "
                      "Butterworth 1.2-30 Hz, sosfiltfilt), empty / noisy trace imputation, per-trace L2 norm"),
    "sliding": dict(kind="sliding", config="configs[3]", n_total=12544, n_ch=4096, n_t=8192, pool=256, pivot_every=8,
                    half_aperture=200.0, gen_chunk=2, merge=49,
                    desc="configs[3]: synthetic passes x 4096 ch x 8192, sliding pivots every 8 channels (+-200 m, "
                         "49 rows), each pass imaged at every pivot it crosses inside its window and its whole window "
                         "validated (||data||_F: NaN / inf / all zero); 12,544 passes per GPU (100k over 8) as 49 "
                         "batches over a resident pool of 256 windows; speed classes x pivots stacked, f-v image per "
                         "(class, pivot)"),
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def tercile_slots(speeds):
    """Exact speed terciles (equal-as-possible class sizes)."""
    slots = np.empty(speeds.size, dtype=np.int64)
    slots[np.argsort(speeds, kind="stable")] = np.arange(speeds.size) * 3 // speeds.size
    return slots


class Batch:
    """One launch's worth of passes: the device plan (tables derived in the step), the class
    schedule, the launch view of the windows and its validity / scale buffers."""

    def __init__(self, plan, sched, win, sumsq, scales, derive=True, validity=True):
        self.plan, self.sched, self.win, self.sumsq, self.scales = plan, sched, win, sumsq, scales
        self.derive, self.validity = derive, validity


class Job:
    """Everything one rank launches per step: batches, class stacks, the f-v chain."""

    def finish(self, n_slot, R, w, gx, dt, device):
        self.stack = torch.zeros((n_slot, R, w), dtype=torch.float32, device=device)
        self.work = torch.empty(max(b.plan.n_pass for b in self.batches) + 2, dtype=torch.int32, device=device)
        s = int(np.abs(gx - (-200.0)).argmin())
        e = int(np.abs(gx - 0.0).argmin())
        self.disp_rows = (s, e + 1)
        self.disp = DispPlan(e + 1 - s, w, 8.16, dt, np.arange(0.8, 25, 0.1), np.arange(200, 1200))
        self.fv = torch.empty((n_slot, self.disp.nV, self.disp.nF), dtype=torch.float32, device=device)


def build_pool(wl, device, world, rank, scaling, chunk):
    """configs[2]: a resident pool of windows, batches of `pool` passes with their own trajectories."""
    job = Job()
    pivot, start_x, end_x = wl["pivot"]
    n_ch, n_t = wl["n_ch"], wl["n_t"]
    # the job's passes of this rank (below) cut into equal batches of at most ~1.05 x the nominal pool, so that no
    # launch carries a remainder of a few passes (strong scaling: 5 120 per rank at N = 2 -> 10 x 512)
    n_loc_pre = wl["n_total"] if scaling != "strong" else shard_passes(np.zeros(wl["n_total"], np.int64), world, rank).size
    n_bat = max(1, -(-n_loc_pre // int(wl["pool"] * 1.05)))
    pool = -(-n_loc_pre // n_bat) if n_loc_pre else wl["pool"]
    t0 = time.time()
    job.windows, x_axis, t_axis, _, _ = synth_batch_device(pool, n_ch=n_ch, n_t=n_t, pivot=pivot, seed=1000 * rank + 3,
                                                           t0=wl.get("t0", DT_W500),
                                                           device=device, x_first=wl["x_first"], track_half=10,
                                                           chunk=wl["gen_chunk"])
    job.t_gen = time.time() - t0
    # the job's passes: speeds 15-30 m/s, pivot crossing within +-1 s of mid-window, on the 1 m / 50 Hz
    # tracking grid.  weak: each rank its own job (seeded by rank); strong: one global job, sharded.
    seed = 7 if scaling == "strong" else 1000 * rank + 7
    rng = np.random.default_rng(seed)
    n_job = wl["n_total"]
    speeds = rng.uniform(15.0, 30.0, n_job)
    tcs = t_axis[n_t // 2] + rng.uniform(-1.0, 1.0, n_job)
    slots = tercile_slots(speeds)
    if scaling == "strong":
        mine = shard_passes(slots, world, rank)
        counts = np.bincount(slots, minlength=3)
    else:
        mine = np.arange(n_job)
        counts = np.bincount(slots, minlength=3) * world  # every rank has the same class sizes
    xs = np.arange(np.floor(pivot) - wl["track_half"], np.floor(pivot) + wl["track_half"] + 1, 1.0)
    t0 = time.time()
    prm = VsgParams(pivot=pivot, start_x=start_x, end_x=end_x, wlen=2, norm=False, include_other_side=True)
    n_loc = mine.size
    assert n_loc == n_loc_pre, (n_loc, n_loc_pre)
    trk_t = torch.empty((n_loc, xs.size), dtype=torch.float64, device=device)
    for b in range(0, n_loc, 1024):  # trajectories to the device in slices (bounded host memory)
        idx = mine[b:b + 1024]
        tt = np.round((tcs[idx, None] + (xs[None, :] - pivot) / speeds[idx, None]) / TRACK_DT) * TRACK_DT
        trk_t[b:b + idx.size].copy_(torch.from_numpy(tt))
    trk_x = torch.from_numpy(xs).to(device).expand(n_loc, xs.size).contiguous()
    trk_len = torch.full((n_loc,), xs.size, dtype=torch.int32, device=device)
    job.sumsq = torch.empty(pool, dtype=torch.float64, device=device)
    # a scale buffer per batch: the step forms every batch's scales up front, side by side on a few streams
    job.scales = torch.empty((n_loc, 2), dtype=torch.float32, device=device)
    job.side_streams = [torch.cuda.Stream(device=device) for _ in range(3)]
    # the step's tables for all its passes in one geometry launch (10 240 blocks instead of 20 launches of
    # 512); each batch's plan is a slice of it
    job.plan_all = DevicePlan(x_axis, t_axis, trk_x, trk_t, trk_len, prm, n_ch, derive=False) if n_loc else None
    job.batches = []
    for b in range(0, n_loc, pool):
        sl = slice(b, min(b + pool, n_loc))
        nb = sl.stop - sl.start
        sched = StackSchedule(slots[mine[sl]], 3, chunk=chunk, counts=counts)
        job.batches.append(Batch(job.plan_all.slice(sl.start, sl.stop), sched, job.windows[:nb], job.sumsq[:nb],
                                 job.scales[sl], derive=False))
        job.batches[-1].slots = slots[mine[sl]]
    job.t_plan = time.time() - t0
    job.n_local, job.n_global = n_loc, (n_job if scaling == "strong" else n_job * world)
    job.units = n_loc
    job.prm, job.x_axis, job.t_axis = prm, x_axis, t_axis
    # host copies of a few passes for the CPU baseline (the reference loop takes host arrays)
    job.cpu_sets = [dict(win=job.windows, x_axis=x_axis, t_axis=t_axis, prm=prm, n_total=job.n_global,
                         trk=[(xs, np.round((tcs[i] + (xs - pivot) / speeds[i]) / TRACK_DT) * TRACK_DT) for i in mine[:64]])]
    R, w = job.batches[0].plan.R, job.batches[0].plan.w
    st, pv = int(np.argmax(x_axis >= start_x)), int(np.argmax(x_axis >= pivot))
    job.finish(3, R, w, x_axis[st:st + R] - x_axis[pv], t_axis[1] - t_axis[0], device)
    return job


def build_resident(wl, device, world, rank, scaling, chunk):
    """configs[0]/[1]: every pass of every pivot set resident in ONE window buffer, one launch."""
    job = Job()
    n_ch, n_t = wl["n_ch"], wl["n_t"]
    sets = wl["pivots"]
    # the job: per pivot set its class labels (seeded identically on every rank for strong scaling)
    slots_g, set_g = [], []
    for i, (_, _, _, counts) in enumerate(sets):
        rng = np.random.default_rng(100 + i if scaling == "strong" else 1000 * rank + 100 + i)
        slots_g.append(rng.permutation(np.repeat(np.arange(len(counts)), counts)) + 3 * i)
        set_g.append(np.full(int(sum(counts)), i))
    slots_g, set_g = np.concatenate(slots_g), np.concatenate(set_g)
    n_slot = 3 * len(sets)
    if scaling == "strong":
        mine = shard_passes(slots_g, world, rank)
        counts = np.bincount(slots_g, minlength=n_slot)
    else:
        mine = np.arange(slots_g.size)
        counts = np.bincount(slots_g, minlength=n_slot) * world
    n = mine.size
    job.windows = torch.empty((n, n_ch, n_t), dtype=torch.float32, device=device)
    t0 = time.time()
    x_axes = np.empty((n, n_ch))
    trks, piv, sx, ex, job.cpu_sets = [], np.empty(n), np.empty(n), np.empty(n), []
    o = 0
    for i, (pivot, start_x, end_x, _) in enumerate(sets):
        k = int(np.sum(set_g[mine] == i))
        if k == 0:
            continue
        _, x_axis, t_axis, trk, _ = synth_batch_device(k, n_ch=n_ch, n_t=n_t, pivot=pivot, seed=1000 * rank + 17 * i + 3,
                                                       t0=wl.get("t0", DT_W500),
                                                       device=device, track_half=wl["track_half"],
                                                       chunk=wl["gen_chunk"], out=job.windows[o:o + k])
        x_axes[o:o + k], piv[o:o + k], sx[o:o + k], ex[o:o + k] = x_axis, pivot, start_x, end_x
        trks += trk
        job.cpu_sets.append(dict(win=job.windows[o:o + k], x_axis=x_axis, t_axis=t_axis, trk=trk[:64],
                                 prm=VsgParams(pivot=pivot, start_x=start_x, end_x=end_x, wlen=2, norm=False,
                                               include_other_side=True),
                                 n_total=int(np.sum(set_g == i)) * (1 if scaling == "strong" else world)))
        o += k
    job.t_gen = time.time() - t0
    t0 = time.time()
    slots_l = slots_g[mine]  # `mine` is ascending and set-major: buffer order
    from das_diff_veh_amd.plan import pack_trajectories
    prm = job.cpu_sets[0]["prm"]
    plan = DevicePlan(x_axes, t_axis, *pack_trajectories(trks, device), prm, n_ch, pivot_x=piv, start_x=sx, end_x=ex,
                      derive=False)
    sched = StackSchedule(slots_l, n_slot, chunk=chunk, counts=counts)
    job.sumsq = torch.empty(n, dtype=torch.float64, device=device)
    job.scales = torch.empty((n, 2), dtype=torch.float32, device=device)
    job.batches = [Batch(plan, sched, job.windows, job.sumsq, job.scales)]
    job.batches[0].slots = slots_l
    job.t_plan = time.time() - t0
    job.n_local = n
    job.n_global = slots_g.size if scaling == "strong" else slots_g.size * world
    job.units = n
    pv0 = int(np.argmax(x_axes[0] >= piv[0]))
    st0 = int(np.argmax(x_axes[0] >= sx[0]))
    job.finish(n_slot, plan.R, plan.w, x_axes[0, st0:st0 + plan.R] - x_axes[0, pv0], t_axis[1] - t_axis[0], device)
    return job


def build_sliding(wl, device, world, rank, scaling, chunk):
    """configs[3]: a pool of long-fiber windows imaged at sliding pivots (UnitPlan, host tables).

    Every batch gives the pool new per-pass trajectories (crossing point uniform along the fiber,
    15-30 m/s, crossing at mid-window), i.e. each batch is `pool` new passes over the resident window
    contents; a pass becomes one unit per pivot it crosses inside its window.  Slots = speed class x
    pivot with fixed class edges (20, 25 m/s); class means use the GLOBAL unit count per slot (one
    all-reduce of the counts at setup).  The batches merge into launches of `merge` batches, and every
    launch validates the windows of all its passes (UnitScan: window per (batch, pass), 134 MB each, read
    once per pass however many pivots it is imaged at): the reference divides a pass's window by
    ||data||_F in every VirtualShotGather call (apis/virtual_shot_gather.py:125)."""
    from das_diff_veh_amd.plan import UnitPlan, sliding_pivots
    from das_diff_veh_amd.vsg import UnitScan, flat_units
    job = Job()
    n_ch, n_t, pool = wl["n_ch"], wl["n_t"], wl["pool"]
    t0 = time.time()
    job.windows, x_axis, t_axis, _, _ = synth_batch_device(pool, n_ch=n_ch, n_t=n_t, pivot=n_ch * 8.16 / 2,
                                                           seed=1000 * rank + 3, device=device, x_first=0.37,
                                                           track_half=10, chunk=wl["gen_chunk"])
    job.t_gen = time.time() - t0
    t0 = time.time()
    prm = VsgParams(wlen=2, norm=False, include_other_side=True)
    edge = 4 * wl["pivot_every"]
    pch = np.arange(edge, n_ch - edge, wl["pivot_every"])
    n_piv = pch.size
    n_total = wl["n_total"] if scaling == "weak" else -(-wl["n_total"] // world)
    rng = np.random.default_rng(1000 * rank + 7)
    n_batch = -(-int(n_total) // pool)
    plans, slot_l, trks = [], [], []
    for _ in range(n_batch):
        x0 = rng.uniform(x_axis[edge], x_axis[-edge], pool)
        v = rng.uniform(15.0, 30.0, pool)
        tc = t_axis[n_t // 2] + rng.uniform(-1.0, 1.0, pool)
        trk = []
        for xa, va, ta in zip(x0, v, tc):
            xs = np.arange(np.floor(xa) - 800.0, np.floor(xa) + 801.0)
            trk.append((xs, np.round((ta + (xs - xa) / va) / TRACK_DT) * TRACK_DT))
        plan = UnitPlan.sliding(x_axis, t_axis, trk, pch, wl["half_aperture"], prm)
        plans.append(plan)
        trks.append(trk)
        slot_l.append(np.digitize(v[plan.unit_window], [20.0, 25.0]) * n_piv + plan.unit_pivot)
    n_slot = 3 * n_piv
    counts = np.bincount(np.concatenate(slot_l), minlength=n_slot)
    if world > 1:
        ct = torch.as_tensor(counts, dtype=torch.int64, device=device)
        allreduce_stacks([ct])
        counts = ct.cpu().numpy()
    # batches of new trajectories over the same pool merge into launches of `merge` batches each: one
    # class (x pivot) slot then holds tens of units per launch instead of ~0.4, so a chunk's inverse
    # transform and stack atomics are shared by up to `chunk` units
    merge = max(1, int(wl.get("merge", 1)))
    job.batches = []
    for m0 in range(0, len(plans), merge):
        grp = plans[m0:m0 + merge]
        plan = UnitPlan.concat(grp) if len(grp) > 1 else grp[0]
        sl = np.concatenate(slot_l[m0:m0 + merge])
        b = Batch(plan, StackSchedule(sl, n_slot, chunk=chunk, counts=counts), flat_units(job.windows, plan), None,
                  torch.empty((plan.n_pass, 2), dtype=torch.float32, device=device), derive=False, validity=True)
        b.scan = UnitScan(np.tile(np.arange(pool) * n_ch, len(grp)),
                          np.concatenate([p.unit_window + k * pool for k, p in enumerate(grp)]), n_ch)
        b.scan_bytes = 4 * b.scan.n_win * n_ch * n_t
        b.slots, b.first_batch, b.n_merged = sl, m0, len(grp)
        job.batches.append(b)
    job.units = sum(p.n_pass for p in plans)
    job.n_local = n_batch * pool
    job.n_global = job.n_local * world
    job.t_plan = time.time() - t0
    job.cpu_sets = None
    job.cpu_units = dict(x_axis=x_axis, t_axis=t_axis, pch=pch, trk=trks[0], plan=plans[0],
                         half=wl["half_aperture"], units_per_pass=job.units / job.n_local)
    job.plans, job.trks = plans, trks  # per batch of trajectories (host bookkeeping; tests/test_bench_job_gpu.py)
    R, w = plans[0].R, plans[0].w
    pv, st, en, _ = sliding_pivots(x_axis, pch[:1], wl["half_aperture"])
    job.finish(n_slot, R, w, x_axis[st[0]:en[0]] - x_axis[pv[0]], t_axis[1] - t_axis[0], device)
    job.work = torch.empty(max(max(b.plan.n_pass, b.scan.n_win) for b in job.batches) + 2, dtype=torch.int32,
                           device=device)
    return job


def build(workload, device, world, rank, scaling="weak", chunk=8):
    wl = WORKLOADS[workload]
    fn = {"pool": build_pool, "resident": build_resident, "sliding": build_sliding}[wl["kind"]]
    return fn(wl, device, world, rank, scaling, chunk)


PHASES = ("geometry", "validity", "scales", "stack")


def step(job, world, ev=None, fused=True):
    """One step; ev (optional) = {phase: list of [start, end] events, one pair per batch}.  fused: the
    windows' validity inside the stack launch (vsg_stack_validated); else a window_sumsq launch per
    batch before the scales."""
    def mark(name, j, k):
        if ev is not None:
            ev[name][j][k].record()
    side = getattr(job, "side_streams", None)
    if side and fused and getattr(job, "plan_all", None) is not None and \
            all(b.validity and (b.plan.flags & 6) and not b.derive for b in job.batches):
        # every batch's tables in one launch, then every batch's scales (one wave per pass, latency bound)
        # spread over the main and side streams so they run side by side, then the stack launches
        main = torch.cuda.current_stream()
        mark("geometry", 0, 0)
        job.plan_all.derive()
        mark("geometry", 0, 1)
        streams = [main] + side
        for st in side:
            st.wait_stream(main)
        mark("scales", 0, 0)  # the phase is the main stream's wall time from the first scales to the join
        for j, b in enumerate(job.batches):
            with torch.cuda.stream(streams[j % len(streams)]):
                vsg_scales(b.win, b.plan, out=b.scales, win_sumsq=None, validity=False)
        for st in side:
            main.wait_stream(st)
        mark("scales", 0, 1)
        for j, b in enumerate(job.batches):
            for name in (("geometry", "validity", "scales") if j > 0 else ("validity",)):
                mark(name, j, 0)
                mark(name, j, 1)
            mark("stack", j, 0)
            vsg_stack_validated(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=j > 0, work=job.work)
            mark("stack", j, 1)
        if world > 1:
            allreduce_stacks([job.stack])
        a, e = job.disp_rows
        fv_from_fk(fk_grid(job.stack[:, a:e, :], job.disp), job.disp, out=job.fv)
        return
    for j, b in enumerate(job.batches):
        mark("geometry", j, 0)
        if j == 0 and getattr(job, "plan_all", None) is not None:
            job.plan_all.derive()  # every batch's tables (the batches' plans are slices of it)
        if b.derive:
            b.plan.derive()
        mark("geometry", j, 1)
        fuse = fused and b.validity and (b.plan.flags & 6)
        mark("validity", j, 0)
        if b.validity and not fuse:
            window_sumsq(b.win, out=b.sumsq)
        mark("validity", j, 1)
        mark("scales", j, 0)
        vsg_scales(b.win, b.plan, out=b.scales, win_sumsq=None if fuse else b.sumsq, validity=not fuse)
        mark("scales", j, 1)
        mark("stack", j, 0)
        if fuse:
            vsg_stack_validated(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=j > 0, work=job.work,
                                scan=getattr(b, "scan", None))
        else:
            vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=j > 0)
        mark("stack", j, 1)
    if world > 1:
        allreduce_stacks([job.stack])
    a, e = job.disp_rows
    fv_from_fk(fk_grid(job.stack[:, a:e, :], job.disp), job.disp, out=job.fv)


def host_cores():
    """The host cores this process may use: the affinity mask and, where a cgroup caps the CPU time (the GPU box
    gives each GPU a share of a large machine), the cap in whole cores.  `usable` = the smaller; the all-core
    CPU-baseline legs start that many single-threaded workers."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):  # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, -(-q // per))
        except (OSError, ValueError):
            pass
    usable = min(aff, quota) if quota else aff
    return {"affinity": aff, "cgroup_quota_cores": quota, "usable": usable, "os_cpu_count": os.cpu_count()}


def run_cpu_workers(kind, arrays, params, budget_s, workers):
    """`workers` single-threaded processes of oracle/cpu_legs.py KIND (no GPU state), all at once for budget_s
    each, over a sample saved as memory-mapped .npy files; returns their result dicts (a worker that fails or
    hangs does not count)."""
    import tempfile
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    res = []
    with tempfile.TemporaryDirectory() as d:
        for k, v in arrays.items():
            np.save(os.path.join(d, k + ".npy"), np.ascontiguousarray(v))
        with open(os.path.join(d, "params.json"), "w") as fh:
            json.dump(params, fh)
        procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_legs", kind, d, str(w), str(budget_s)], cwd=ROOT,
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                 for w in range(workers)]
        for pr in procs:
            try:
                out, _ = pr.communicate(timeout=budget_s * 6 + 180)
                res.append(json.loads(out.strip().splitlines()[-1]))
            except Exception:
                pr.kill()
    if not res:
        raise RuntimeError(f"no CPU-baseline worker ({kind}) finished")
    return res


def cpu_baseline(job, budget_s=20.0, workers=None):
    """Reference-structured CPU path (oracle/ref_loop.py) on a bounded sample of the same windows.

    1 core: the bench windows themselves (host copies) for about budget_s / 2, plus one f-v image per pivot set.
    All cores: one single-threaded process per usable host core (host_cores(): affinity mask, cgroup cap), each
    looping over a saved sample of the windows for budget_s / 2 and then imaging its stack (oracle/cpu_legs.py
    vsg); windows/s and images/s are both measured with every core busy, and the step's windows and class images
    are priced at those aggregate rates."""
    from oracle import ref_loop
    torch.set_num_threads(1)
    cores = host_cores()
    workers = workers or cores["usable"]
    n_win, t_win, t_img, n_img = 0, 0.0, 0.0, 0
    t_start = time.time()
    one_budget = budget_s / 2
    samples = []
    for s in job.cpu_sets:
        x_axis, t_axis, trk, prm, win = s["x_axis"], s["t_axis"], s["trk"], s["prm"], s["win"]
        wbytes = 8 * win[0].numel()
        k = min(len(trk), win.shape[0], max(2, int(2e9 / wbytes)))  # host copy <= 2 GB
        host = win[:k].to("cpu", torch.float64).numpy()
        ns = max(2, min(16, k, int(256e6 / (wbytes / 2))))  # worker sample <= 256 MB of float32
        samples.append((host[:ns].astype(np.float32), x_axis, t_axis, trk[:ns], prm))
        t0 = time.time()
        acc = None
        done = 0
        for i in range(k):
            g, gx, gt = ref_loop.gather(host[i], x_axis, t_axis, trk[i][0], trk[i][1], prm.pivot, prm.start_x,
                                        prm.end_x)
            acc = g if acc is None else acc + g
            done += 1
            if time.time() - t_start > one_budget:
                break
        t_win += time.time() - t0
        n_win += done
        t0 = time.time()
        ref_loop.disp_image(acc / done, gx, gt)
        t_img += time.time() - t0
        n_img += 1
    per_window = t_win / n_win
    per_image = t_img / n_img
    total_windows = sum(s["n_total"] for s in job.cpu_sets)
    total_images = job.stack.shape[0]
    rate1 = total_windows / (per_window * total_windows + per_image * total_images)
    host, x_axis, t_axis, trk, prm = samples[0]
    res = run_cpu_workers("vsg", dict(wins=host, x_axis=x_axis, t_axis=t_axis, vx=np.stack([v for v, _ in trk]),
                                      vt=np.stack([t for _, t in trk])),
                          dict(pivot=prm.pivot, start_x=prm.start_x, end_x=prm.end_x), budget_s / 2, workers)
    win_rate = sum(r["windows"] / r["secs"] for r in res)
    img_rate = sum(r["images"] / r["img_secs"] for r in res)
    step_s = total_windows / win_rate + total_images / img_rate
    return dict(value=total_windows / step_s, unit="vehicle-pass windows/s", cores=len(res), kind="port",
                host_cores=cores,
                sample=f"all cores: {len(res)} single-threaded processes (usable cores: affinity {cores['affinity']}, "
                       f"cgroup cap {cores['cgroup_quota_cores']}), each {budget_s / 2:.0f} s of VSG gathers over "
                       f"{host.shape[0]} saved windows ({sum(r['windows'] for r in res)} windows, two-sided) then f-v "
                       f"images of its stack ({sum(r['images'] for r in res)} images), both rates measured with every "
                       f"core busy: {win_rate:.2f} windows/s, {img_rate:.1f} images/s; 1 core: {n_win} windows "
                       f"({per_window * 1e3:.1f} ms/window), {n_img} f-v images ({per_image * 1e3:.1f} ms/image) -> "
                       f"{rate1:.2f} windows/s; the port leaves out the reference's per-__add__ deepcopy of the window "
                       f"(apis/virtual_shot_gather.py:196), so the reference itself is slower; "
                       f"cpu={platform.processor() or platform.machine()}",
                value_1core=rate1)


def cpu_baseline_sliding(job, budget_s=20.0, workers=None):
    """configs[3] CPU path: oracle/ref_loop.gather (the reference's VirtualShotGather loop, including its
    data / ||data||_F of the whole 4,096 x 8,192 window per call) for sample units of the bench's first
    batch, each at its own pivot (start_x / end_x = pivot -/+ 200 m), on host copies of their windows.
    1 core over the sample for budget_s / 2, then one single-threaded process per usable host core for budget_s / 2
    (oracle/cpu_legs.py vsg: units, then f-v images of the worker's stack, both measured with every core busy);
    passes/s = units/s / (units per pass), with the step's images at the measured aggregate image rate."""
    from oracle import ref_loop
    torch.set_num_threads(1)
    cores = host_cores()
    workers = workers or cores["usable"]
    cu = job.cpu_units
    x_axis, t_axis, pch, trk, plan, half = (cu[k] for k in ("x_axis", "t_axis", "pch", "trk", "plan", "half"))
    ns = min(4, plan.n_pass)
    units = list(range(ns))
    hosts = {}
    for u in units:
        q = int(plan.unit_window[u])
        if q not in hosts:
            hosts[q] = job.windows[q].to("cpu", torch.float64).numpy()
    t_start, n_u, t_u, acc, ax = time.time(), 0, 0.0, None, None
    while time.time() - t_start < budget_s / 2:
        u = units[n_u % ns]
        q, p = int(plan.unit_window[u]), float(x_axis[pch[int(plan.unit_pivot[u])]])
        t0 = time.time()
        g, gx, gt = ref_loop.gather(hosts[q], x_axis, t_axis, trk[q][0], trk[q][1], p, p - half, p + half)
        t_u += time.time() - t0
        n_u += 1
        acc, ax = g, (gx, gt)
    t0 = time.time()
    ref_loop.disp_image(acc, *ax)
    per_image = time.time() - t0
    per_unit = t_u / n_u
    upp = cu["units_per_pass"]
    n_img = job.stack.shape[0]
    rate1 = job.n_global / (per_unit * upp * job.n_global + per_image * n_img)
    qs = [int(plan.unit_window[u]) for u in units]
    pv = np.array([float(x_axis[pch[int(plan.unit_pivot[u])]]) for u in units])
    res = run_cpu_workers("vsg", dict(wins=np.stack([hosts[q].astype(np.float32) for q in qs[:2]]), x_axis=x_axis,
                                      t_axis=t_axis, vx=np.stack([trk[q][0] for q in qs[:2]]),
                                      vt=np.stack([trk[q][1] for q in qs[:2]]), pivot=pv[:2], start_x=pv[:2] - half,
                                      end_x=pv[:2] + half), {}, budget_s / 2, workers)
    unit_rate = sum(r["windows"] / r["secs"] for r in res)
    img_rate = sum(r["images"] / r["img_secs"] for r in res)
    step_s = job.n_global * upp / unit_rate + n_img / img_rate
    return dict(value=job.n_global / step_s, unit="vehicle-pass windows/s", cores=len(res), kind="port",
                host_cores=cores,
                sample=f"all cores: {len(res)} single-threaded processes (usable cores: affinity {cores['affinity']}, "
                       f"cgroup cap {cores['cgroup_quota_cores']}) x {budget_s / 2:.0f} s, "
                       f"{sum(r['windows'] for r in res)} (pass, pivot) units of 2 saved 4,096 x 8,192 windows (VSG "
                       f"two-sided, +-{half:.0f} m at each unit's pivot), then f-v images of each worker's stack "
                       f"({sum(r['images'] for r in res)}), both rates with every core busy: {unit_rate:.2f} units/s, "
                       f"{img_rate:.1f} images/s; {upp:.2f} units per pass; 1 core: {n_u} units "
                       f"({per_unit * 1e3:.0f} ms/unit, the window's data / ||data|| included), f-v image "
                       f"{per_image * 1e3:.1f} ms -> {rate1:.3f} passes/s; without the reference's per-__add__ deepcopy "
                       f"(apis/virtual_shot_gather.py:196); cpu={platform.processor() or platform.machine()}",
                value_1core=rate1)


def layout_of(job, args, scaling):
    """What one profiled launch of the stack kernel covers (PMC counters are per launch)."""
    lay = {"workload": args.workload, "chunk": args.chunk, "scaling": scaling,
           "validity": "separate" if args.separate_validity else "fused",
           "passes_per_launch": [int(b.plan.n_pass) for b in job.batches][:1],
           "launches_per_step": len(job.batches)}
    if job.batches[0].plan.w != 500:
        lay["w"] = int(job.batches[0].plan.w)
    return lay


def pmc_lookup(kernel, layout, key):
    """Per-launch value of `key` for `kernel` from the newest committed PMC summary whose recorded
    launch layout equals this run's.  (None, note) when no summary matches: counters of a different
    launch shape divided by this run's launch time would be wrong by the ratio of the shapes."""
    sfx = "" if layout["workload"] == "synth10k" else "_" + layout["workload"]
    if "w" in layout:  # tools/pmc.sh <tag> w499 | weights_w499
        sfx = f"_w{layout['w']}" if layout["workload"] == "synth10k" else f"{sfx}_w{layout['w']}"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_summary{sfx}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("layout") != layout:
            continue
        if kernel in d and key in d[kernel]:
            return float(d[kernel][key]), os.path.basename(f)
    return None, "no committed PMC summary with this launch layout"


# FP64 matrix peak: MI355X_MICROARCH.md has no FP64 MFMA row; the spec sheet's 78.6 TF is not reached by
# v_mfma_f64_16x16x4_f64 on this box: tools/calib/dp_pipes measures 47.0-47.8 TF with 2-4 waves per SIMD
# (profiles/r2g_dp_pipes.txt), the measured ceiling used as `peak` (the spec figure is reported beside it)
FP64_MFMA_PEAK_TF = 47.8
FP64_MFMA_SPEC_TF = 78.6


def timelapse_main(args, world, rank, device):
    """configs[4]: one step = the f-v images of B resident gathers (tdft + fk contraction + f-v kernels,
    the product dispatch).  Days shard over the ranks with no data-path collective (weak scaling).
    Roofline of the dominant kernel (the MFMA f-v kernel): float64 MFMA FLOPs it issues per launch / the
    launch's HIP-event time on its stream, and the HBM fraction of the f-v bytes it writes."""
    from das_diff_veh_amd import _lib
    from das_diff_veh_amd.disp import _use_mfma
    from das_diff_veh_amd.synth import synth_gathers
    wl = WORKLOADS["timelapse"]
    B, nch, nt = wl["B"], wl["nch"], wl["nt"]
    dx, dt = 8.16, 0.003999999999997783
    freqs, vels = np.linspace(1.0, 25.0, wl["nF"]), np.linspace(200.0, 1200.0, wl["nV"])
    t0 = time.time()
    plan = DispPlan(nch, nt, dx, dt, freqs, vels)
    data = synth_gathers(B, nch, nt, dx, dt, device, seed=1000 + rank)
    tb = plan.tables(device)
    st = _lib.stream_of(device)
    stream = torch.cuda.current_stream(device)
    D = torch.empty((B * nch, 2 * plan.n_fb), dtype=torch.float64, device=device)
    FK = torch.empty((B, plan.n_kb, plan.n_fb), dtype=torch.float64, device=device)
    fv = torch.empty((B, plan.nV, plan.nF), dtype=torch.float32, device=device)
    t_setup = time.time() - t0

    def run(ev=None):
        if ev:
            ev[0].record(stream)
        _lib.call("dvh_disp_tdft", _lib.ptr(data), data.stride(0), data.stride(1), B, nch, nt, _lib.ptr(tb["wt"]),
                  plan.n_fb, None, _lib.ptr(D), st)
        if ev:
            ev[1].record(stream)
        _lib.call("dvh_disp_fk", _lib.ptr(D), B, nch, plan.n_fb, _lib.ptr(tb["atab"]), plan.MT, plan.K2, plan.n_kb,
                  _lib.ptr(FK), None, None, 0, st)
        if ev:
            ev[2].record(stream)
        fv_from_fk(FK, plan, out=fv)
        if ev:
            ev[3].record(stream)

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        run(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)
    t = np.array([[e[i].elapsed_time(e[i + 1]) for i in range(3)] for e in evs]).mean(axis=0) / 1e3  # s

    # parity: two images against the oracle (after timing)
    from oracle import disp as odisp
    host = data.double().cpu().numpy()
    errs, picks = [], []
    for b in (0, B - 1):
        ref = odisp.map_fv(host[b], dx, dt, freqs, vels)
        got = fv[b].double().cpu().numpy()
        errs.append(float(np.abs(got - ref).max() / np.abs(ref).max()))
        picks.append(bool(np.all(odisp.pick_ok(ref, got.argmax(axis=0)))))

    mfma = _use_mfma(plan, B)
    n_tiles = -(-(plan.nF - 16) // 16) + 1
    mfma_flop = 2.0 * 16 * 16 * 40 * n_tiles * B * -(-plan.nV // 16)  # 10 v_mfma_f64_16x16x4 per 16 x 16 tile
    fv_bytes = 4.0 * B * plan.nV * plan.nF + 8.0 * B * plan.n_kb * plan.n_fb
    tdft_flop = 2.0 * B * nch * nt * 2 * plan.n_fb
    traffic, traffic_src = None, "no committed time-lapse PMC summary"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary_timelapse.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        k = d.get("fv_mfma_kernel")
        if mfma and k and "traffic_bytes" in k and (B, plan.nV, plan.nF) == (512, 512, 1000):
            traffic, traffic_src = float(k["traffic_bytes"]), os.path.basename(f)  # tools/pmc_timelapse.sh: same shape
            break
    achieved = (mfma_flop if mfma else 2.0 * 25 * B * plan.nV * plan.nF) / t[2] / 1e12
    res = {
        "metric": "time-lapse f-v images/sec (configs[4]: 512 velocities x 1,000 frequencies per image); % MFMA roofline",
        "value": world * B * args.steps / elapsed, "unit": "f-v images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64 (DFT, contraction, FIR on the MFMA pipe), f32 images",
        "data": "synthetic dispersive gathers (c(f) = 250 + 4000 / (f + 4) m/s + noise), resident",
        "config": {"workload": "timelapse", "baseline_config": wl["config"], "description": wl["desc"],
                   "gathers_per_step_this_rank": B, "nch": nch, "nt": nt, "nV": plan.nV, "nF": plan.nF,
                   "parallelism": f"dp{world} (days sharded, no exchange)"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_SPEC_TF, "unit": "TFLOP/s",
                     "frac": achieved / FP64_MFMA_SPEC_TF, "traffic": traffic, "traffic_source": traffic_src,
                     "peak_source": "MI355X spec sheet FP64 matrix 78.6 TF; a v_mfma_f64_16x16x4_f64 loop measures "
                                    "47.8 TF on the box (tools/calib/dp_pipes, profiles/r2g_dp_pipes.txt)",
                     "frac_of_measured_ceiling": achieved / FP64_MFMA_PEAK_TF,
                     "kernel": "fv_mfma_kernel" if mfma else "fv_tile_kernel", "launch_ms": t[2] * 1e3,
                     "flop_model": "10 v_mfma_f64_16x16x4_f64 per (16 velocities x 16 frequencies) tile, "
                                   "ceil((nF - 16) / 16) + 1 tiles per row" if mfma else "25-tap FIR",
                     "hbm_bytes_per_launch": fv_bytes, "hbm_frac": fv_bytes / t[2] / 1e9 / HBM_PEAK_GBS},
        "kernels_ms": {"time_dft": t[0] * 1e3, "fk_contract": t[1] * 1e3, "fv": t[2] * 1e3},
        "time_dft_mfma_frac": tdft_flop / t[0] / 1e12 / FP64_MFMA_SPEC_TF,
        "time_dft_mfma_frac_of_measured_ceiling": tdft_flop / t[0] / 1e12 / FP64_MFMA_PEAK_TF,
        "parity": {"max_rel_err": max(errs), "picks_ok": all(picks), "images_checked": 2, "tol": 1e-4},
        "host_setup_s": t_setup,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the oracle's map_fv (fft2, FITPACK bilinear via RectBivariateSpline, savgol) on one core over a
        # bounded sample of the same gathers, then on every usable core at once (oracle/cpu_legs.py fv)
        budget = args.cpu_budget / 2
        torch.set_num_threads(1)
        n, t_c = 0, time.time()
        while time.time() - t_c < budget and n < B:
            odisp.map_fv(host[n], dx, dt, freqs, vels)
            n += 1
        secs = time.time() - t_c
        cores = host_cores()
        wres = run_cpu_workers("fv", dict(gathers=host[:16], freqs=freqs, vels=vels), dict(dx=dx, dt=dt), budget,
                               cores["usable"])
        rate = sum(r["images"] / r["secs"] for r in wres)
        res["cpu_baseline"] = {"value": rate, "unit": "f-v images/s", "cores": len(wres), "kind": "port",
                               "host_cores": cores, "value_1core": n / secs,
                               "sample": f"oracle/disp.py map_fv: all cores: {len(wres)} single-threaded processes x "
                                         f"{budget:.0f} s over 16 of the bench gathers ({sum(r['images'] for r in wres)} "
                                         f"images; usable cores: affinity {cores['affinity']}, cgroup cap "
                                         f"{cores['cgroup_quota_cores']}); 1 core: {n} gathers in {secs:.1f} s; "
                                         f"cpu={platform.processor() or platform.machine()}"}
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


FP64_VALU_SPEC_TF = 78.6  # MI355X spec sheet, FP64 vector


def prep_main(args, world, rank, device):
    """one step = _preprocessing_for_surface_waves of a resident continuous record (a new
    tensor each step, as the reference's data.copy()).  Records shard over the ranks (no exchange).
    Roofline of the dominant kernels (dvh_sosfiltfilt's block filters): the sequential sosfiltfilt's
    float64 operations (9 per sample per section, forward and backward over the padded extension) / the
    bandpass' HIP-event time, against the FP64 vector peak; the block-parallel form issues 2x that."""
    from das_diff_veh_amd.preprocess import _design, surface_wave_preprocessing
    wl = WORKLOADS["prep"]
    n_ch, dt = wl["n_ch"], wl["dt"]
    n_t = int(round(wl["seconds"] / dt))
    gen = torch.Generator(device=device)
    gen.manual_seed(77 + rank)
    t = torch.arange(n_t, device=device, dtype=torch.float64) * dt
    rec = (torch.randn((n_ch, n_t), generator=gen, device=device, dtype=torch.float32) * 0.1 +
           torch.sin(2 * np.pi * 7.0 * t)[None, :].float())
    rec[100].zero_()          # an empty trace (imputed from its neighbours)
    rec[333, 5000] = 1e3      # a noisy trace
    sos, padlen, _, _ = _design(dt, 1.2, 30, device)
    n_sec, n_ext = len(sos), n_t + 2 * padlen
    phases = {}

    def run(ph=None):
        return surface_wave_preprocessing(rec, dt, _phases=ph)

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    evs = [{} for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = run(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)
    bp = float(np.mean([e["bandpass0"].elapsed_time(e["bandpass1"]) for e in evs])) / 1e3
    cl = float(np.mean([e["bandpass1"].elapsed_time(e["cleanup1"]) for e in evs])) / 1e3
    flop = 2.0 * 9 * n_sec * n_ext * n_ch  # sequential sosfiltfilt: forward + backward passes
    # dvh_sosfiltfilt's block GEMMs on the float64 matrix pipe (csrc/dvh_prep.hip, 64-sample blocks, 16 blocks per
    # tile, 2 NS = 20 states): forward end states 32, forward outputs (lower-triangular Toeplitz with its zero
    # 16 x 16 tiles skipped, start states) + backward end states 92, backward outputs (upper-triangular) 60
    # v_mfma_f64_16x16x4_f64 per tile
    n_tiles = n_ch * (-(-n_ext // 64)) / 16.0
    mfma_flop = n_tiles * (32 + 92 + 60) * 2.0 * 16 * 16 * 4
    rec_bytes = 4.0 * n_ch * n_t
    # parity (after timing): the step's output against the reference's own path on the whole record
    # (scipy.signal.sosfiltfilt as bandpass_data calls it, then the imputation and norm), and the bandpass
    # of two traces against the oracle's pure-Python sosfiltfilt restatement (pinned by tests/golden/prep.npz)
    from das_diff_veh_amd.preprocess import bandpass_inplace
    from oracle import preprocess as oprep
    host = rec.cpu().numpy()
    ref = oprep.surface_wave_prep(host, dt, scipy_filter=True)
    got = out.double().cpu().numpy()
    err = float(np.abs(got - ref).max() / np.abs(ref).max())
    bp_dev = rec[[0, 700]].double().clone()
    bandpass_inplace(bp_dev, dt, 1.2, 30)
    bp_ref = oprep.bandpass_data(host[[0, 700]], dt, 1.2, 30)
    err_bp = float(np.abs(bp_dev.cpu().numpy() - bp_ref).max() / np.abs(bp_ref).max())
    res = {
        "metric": "continuous-record preprocessing: records/s (_preprocessing_for_surface_waves, 1,024 ch x 60 s); "
                  "% FP64 roofline of the bandpass",
        "value": world * args.steps / elapsed, "unit": "records/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64 recursion, f32 record",
        "data": "synthetic float32 record (7 Hz tone + noise, one empty and one spiky trace), resident",
        "config": {"workload": "prep", "baseline_config": wl["config"], "description": wl["desc"], "n_ch": n_ch,
                   "n_t": n_t, "sections": n_sec, "padlen": padlen, "parallelism": f"dp{world} (records sharded)"},
        "trace_samples_per_s": world * args.steps * n_ch * n_t / elapsed,
        "roofline": {"bound": "fp64-valu", "achieved": flop / bp / 1e12, "peak": FP64_VALU_SPEC_TF, "unit": "TFLOP/s",
                     "frac": flop / bp / 1e12 / FP64_VALU_SPEC_TF, "traffic": None,
                     "kernel": "dvh_sosfiltfilt_planned (sosm_fa / sosm_scanm / sosm_fc / sosm_bf / sosm_scanm / "
                               "sosm_bc: block GEMMs and two-level state scans on the float64 MFMA pipe)",
                     "launch_ms": bp * 1e3, "flop_model": "9 flops per sample per section (scipy sosfilt), forward + "
                                                          "backward over n_t + 2 padlen (the sequential filter's work)",
                     "mfma_flop_issued": mfma_flop, "mfma_achieved_tflops": mfma_flop / bp / 1e12,
                     "mfma_frac_of_spec": mfma_flop / bp / 1e12 / FP64_MFMA_SPEC_TF,
                     "mfma_model": "64-sample blocks as float64 MFMA GEMMs: 184 v_mfma_f64_16x16x4_f64 per 16 blocks "
                                   "(forward end states 32, forward outputs + backward end states 92, backward outputs "
                                   "60); the state scans' own MFMAs (10 per step of 16 groups) not counted",
                     "hbm_bytes_model": "record read + y (f64) written and read + record written",
                     "hbm_frac": (2 * rec_bytes + 16.0 * n_ch * n_ext) / bp / 1e9 / HBM_PEAK_GBS},
        "kernels_ms": {"bandpass": bp * 1e3, "trace_cleanup": cl * 1e3},
        "parity": {"max_rel_err": err, "tol": 2e-6,
                   "reference": "oracle/preprocess.py surface_wave_prep(scipy_filter=True): scipy.signal.sosfiltfilt as "
                                "bandpass_data calls it, imputation and norm in float64, on the whole record",
                   "bandpass_rel_err_vs_restatement": err_bp, "bandpass_tol": 1e-10,
                   "bandpass_check": "traces 0 and 700 in float64 against oracle/preprocess.py's pure-Python sosfiltfilt"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the oracle (scipy's sosfiltfilt + the reference's imputation / norm) on one core, on trace slices of the
        # same record for ~cpu_budget / 2 s, scaled to the full record; then every usable core at once, each worker
        # on its own 64-trace slice (oracle/cpu_legs.py prep)
        torch.set_num_threads(1)
        sub = host[:128]
        n, t_c = 0, time.time()
        while time.time() - t_c < args.cpu_budget / 2 or n < 2:
            oprep.surface_wave_prep(sub, dt, scipy_filter=True)
            n += 1
        secs = (time.time() - t_c) / n
        cores = host_cores()
        wres = run_cpu_workers("prep", dict(record=host[128:192]), dict(dt=dt), args.cpu_budget / 2, cores["usable"])
        rate = sum(r["rows"] / r["secs"] for r in wres) / n_ch
        res["cpu_baseline"] = {"value": rate, "unit": "records/s", "cores": len(wres), "kind": "port",
                               "host_cores": cores, "value_1core": sub.shape[0] / n_ch / secs,
                               "sample": f"the reference's path (scipy.signal.sosfiltfilt as bandpass_data calls it + "
                                         f"oracle/preprocess.py's imputation and norm): all cores: {len(wres)} "
                                         f"single-threaded processes x {args.cpu_budget / 2:.0f} s, each on a 64-trace "
                                         f"slice of the record ({sum(r['rows'] for r in wres)} traces; usable cores: "
                                         f"affinity {cores['affinity']}, cgroup cap {cores['cgroup_quota_cores']}), "
                                         f"traces/s / {n_ch}; 1 core: 128 traces, {n} runs ({secs * 1e3:.0f} ms each), "
                                         f"scaled x {n_ch // 128} to the 1,024-trace record; "
                                         f"cpu={platform.processor() or platform.machine()}"}
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bootstrap_main(args, world, rank, device):
    """one step = the notebook's convergence_test for one class (gathers of the class's
    resident windows, then bt_size 1..60 x 30 resamples through one dispersion batch and 4 ridges).  Classes
    shard over the ranks (no exchange).  Roofline of the dominant kernel (the MFMA f-v kernel over the 1,800
    resample images)."""
    import random

    from das_diff_veh_amd import bootstrap as bt
    from das_diff_veh_amd.disp import _use_mfma
    from das_diff_veh_amd.plan import pack_trajectories
    import scipy.interpolate
    wl = WORKLOADS["bootstrap"]
    n, S, T = wl["n"], wl["max_size"], wl["bt_times"]
    wins, x_axis, t_axis, trk, _ = synth_batch_device(n, pivot=700.0, seed=3 + 1000 * rank, device=device)
    tx, tt, tl = pack_trajectories(trk, device)
    sigma, ref_idx, lb, ub = [25, 50, 50, 50], [80, 130, 170, 170], [2.5, 10, 14, 16], [14, 15, 19, 20]
    curves = [None,
              scipy.interpolate.interp1d([10, 12, 13, 14, 15, 16], [530, 470, 450, 430, 410, 391]),
              scipy.interpolate.interp1d([14, 15, 16, 17, 18, 19], [630, 583, 550, 520, 500, 490]),
              scipy.interpolate.interp1d([16, 17, 18, 19, 20, 21], [745, 690, 657, 626, 600, 580])]

    def run(seed, ph=None):
        if ph is not None:
            ph.setdefault("gather0", torch.cuda.Event(enable_timing=True)).record()
        cache = bt.GatherCache.from_device(wins, x_axis, t_axis, tx, tt, tl, 700.0, 500.0, 900.0)
        return cache, bt.convergence(cache, S, T, sigma, ref_idx, lb, ub, curves, rand=random.Random(seed), phases=ph)

    for k in range(args.warmup):
        run(k)
    torch.cuda.synchronize()
    evs = [{} for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        cache, std = run(100 + k, evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)

    def span(a, b):
        return float(np.mean([e[a].elapsed_time(e[b]) for e in evs])) / 1e3
    t_gather, t_sel, t_disp, t_ridge = span("gather0", "select0"), span("select0", "select1"), \
        span("select1", "disp1"), span("disp1", "ridge1")
    _, _, plan = cache.disp_plan()
    B = S * T
    mfma = _use_mfma(plan, B)
    # the f-v launch alone (dominant kernel): time it on its stream after the timed steps, same batch
    stacks = cache.resample_stacks(np.tile(np.arange(1, 31, dtype=np.int32), (B, 1)))
    FK = bt.fk_grid(stacks, plan)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        bt.fv_from_fk(FK, plan)
    reps = 5
    e0.record()
    for _ in range(reps):
        bt.fv_from_fk(FK, plan)
    e1.record()
    torch.cuda.synchronize()
    t_fv = e0.elapsed_time(e1) / reps / 1e3
    n_tiles = -(-(plan.nF - 16) // 16) + 1
    mfma_flop = 2.0 * 16 * 16 * 40 * n_tiles * B * -(-plan.nV // 16)
    achieved = (mfma_flop if mfma else 2.0 * 25 * B * plan.nV * plan.nF) / t_fv / 1e12
    res = {
        "metric": "bootstrap convergence_test: resamples/s (one class, bt_size 1..60 x 30, 4 ridge modes); % MFMA "
                  "roofline of the f-v kernel",
        "value": world * B * args.steps / elapsed, "unit": "resamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 gathers / stacks, f64 dispersion (MFMA), f32 images",
        "data": "synthetic passes (device-generated moving-source wavefield), resident windows; draws from "
                "random.Random(seed) exactly as the notebook's random.sample",
        "config": {"workload": "bootstrap", "baseline_config": wl["config"], "description": wl["desc"], "passes": n,
                   "resamples_per_step": B, "nV": plan.nV, "nF": plan.nF, "gather_rows_imaged": plan.nch,
                   "parallelism": f"dp{world} (classes sharded)"},
        "step_breakdown_ms": {"gathers_and_host_draws": t_gather * 1e3, "resample_stacks": t_sel * 1e3,
                              "dispersion": t_disp * 1e3, "ridges": t_ridge * 1e3,
                              "host_draws": float(np.mean([e["draw_host_s"] for e in evs])) * 1e3},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_SPEC_TF, "unit": "TFLOP/s",
                     "frac": achieved / FP64_MFMA_SPEC_TF, "frac_of_measured_ceiling": achieved / FP64_MFMA_PEAK_TF,
                     "traffic": None, "kernel": "fv_mfma_kernel" if mfma else "fv_kernel", "launch_ms": t_fv * 1e3,
                     "flop_model": "10 v_mfma_f64_16x16x4_f64 per (16 v x 16 f) tile" if mfma else "25-tap FIR",
                     "hbm_frac": 4.0 * B * plan.nV * plan.nF / t_fv / 1e9 / HBM_PEAK_GBS},
        "std_sum_mode0_first_last": [float(std[0, 0]), float(std[0, -1])],
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the reference's bootstrap_disp recomputes every gather of every resample: its cost per resample of
        # size k is k VSG gathers + one f-v image + 4 ridges; timed with the oracle on one core (gather, f-v
        # image, ridge) on the bench's own windows, then priced over the step's 1,800 resamples
        from oracle import ref_loop
        from oracle import ridge as orid
        torch.set_num_threads(1)
        host = wins[:8].double().cpu().numpy()
        tg, ng, t_c = 0.0, 0, time.time()
        gs = []
        while time.time() - t_c < args.cpu_budget / 3 or ng < 2:
            i = ng % host.shape[0]
            ta = time.time()
            g, gx, gt = ref_loop.gather(host[i], x_axis, t_axis, trk[i][0], trk[i][1], 700.0, 500.0, 900.0)
            tg += time.time() - ta
            ng += 1
            gs.append(g)
        ta = time.time()
        fv = ref_loop.disp_image(np.mean(gs, axis=0), gx, gt, start_x=-150, end_x=0)
        t_img = time.time() - ta
        ta = time.time()
        fq = bt.FREQS
        for m in range(4):
            band = (fq >= lb[m]) & (fq < ub[m])
            try:
                orid.extract_ridge_ref_idx(fq[band], bt.VELS, fv[:, band], ref_freq_idx=ref_idx[m] - int(np.sum(fq < lb[m])),
                                           sigma=sigma[m], vel_max=800, ref_vel=curves[m])
            except ValueError:
                pass
        t_rdg = time.time() - ta
        per_g = tg / ng
        windows_drawn = T * S * (S + 1) // 2
        cpu_s = windows_drawn * per_g + B * (t_img + t_rdg)
        # every usable core at once: each worker prices the same step from its own measured pieces
        cores = host_cores()
        pts = [None] + [[list(map(float, c.x)), list(map(float, c.y))] for c in curves[1:]]
        wres = run_cpu_workers("boot", dict(wins=host.astype(np.float32), x_axis=x_axis, t_axis=t_axis,
                                            vx=np.stack([trk[i][0] for i in range(host.shape[0])]),
                                            vt=np.stack([trk[i][1] for i in range(host.shape[0])])),
                               dict(pivot=700.0, start_x=500.0, end_x=900.0, sigma=sigma, ref_idx=ref_idx, lb=lb, ub=ub,
                                    curves=pts), args.cpu_budget / 2, cores["usable"])
        rate = sum(B / (windows_drawn * r["g_secs"] / r["gathers"] + B * (r["img_secs"] + r["ridge_secs"]))
                   for r in wres)
        res["cpu_baseline"] = {"value": rate, "unit": "resamples/s", "cores": len(wres), "kind": "port",
                               "host_cores": cores, "value_1core": B / cpu_s,
                               "sample": f"oracle, all cores: {len(wres)} single-threaded processes (usable cores: "
                                         f"affinity {cores['affinity']}, cgroup cap {cores['cgroup_quota_cores']}), each "
                                         f"timing VSG gathers for {0.7 * args.cpu_budget / 2:.0f} s "
                                         f"({sum(r['gathers'] for r in wres)} in all), one f-v image and 4 ridges, every "
                                         f"core busy, and pricing the step: {windows_drawn} gathers (the reference "
                                         f"recomputes every resample's gathers) + {B} images + ridges; 1 core: {ng} VSG "
                                         f"gathers ({per_g * 1e3:.1f} ms each, oracle/ref_loop.py), one f-v image "
                                         f"({t_img * 1e3:.1f} ms, map_fv) and 4 ridges ({t_rdg * 1e3:.1f} ms); "
                                         f"cpu={platform.processor() or platform.machine()}"}
        res["speedup_vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_main(args, world, rank, device):
    """The drop-in classes fed from host memory (imaging_diff_speed.ipynb's get_images calls): one step = the
    three classes' get_images on NumPy windows, their H2D staging (device.stage_windows: pinned double
    buffers, thread-parallel host copies, asynchronous copies on a side stream) included.  Bound: PCIe.
    value = windows/s; the roofline is the H2D bandwidth of the step's window bytes."""
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows
    wl = WORKLOADS["speeds-host"]
    n_ch, n_t = wl["n_ch"], wl["n_t"]
    n = sum(wl["classes"])
    dev_w, x_axis, t_axis, trk, _ = synth_batch_device(n, n_ch=n_ch, n_t=n_t, pivot=700.0, seed=5 + 1000 * rank,
                                                       device=device)
    host = dev_w.cpu().numpy()
    del dev_w
    wins = []
    for i in range(n):
        w = SurfaceWaveWindow.__new__(SurfaceWaveWindow)  # the tracked trajectory given directly (no tracker arrays)
        w.data, w.x_axis, w.t_axis = np.ascontiguousarray(host[i]), x_axis, t_axis
        w.veh_state_x, w.veh_state_t = trk[i]
        wins.append(w)
    del host
    cls = np.repeat(np.arange(3), wl["classes"])
    per_class = [[wins[i] for i in np.flatnonzero(cls == c)] for c in range(3)]
    kw = dict(include_other_side=True, pivot=700, start_x=500, end_x=900, wlen=2)

    def run():
        out = []
        for ws in per_class:
            im = VirtualShotGathersFromWindows(ws)
            im.get_images(**kw)
            out.append(im.avg_image.XCF_out)
        return out

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res_imgs = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)
    step_s = elapsed / args.steps
    win_bytes = 4.0 * n * n_ch * n_t
    # the H2D rate of a pinned 64 MB copy on this box (the bound of a host-fed step)
    pin = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(64 << 20, dtype=torch.uint8, device=device)
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    for _ in range(10):
        dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 10 * (64 << 20) / (time.perf_counter() - ta) / 1e9
    res = {
        "metric": "host-fed vehicle-pass windows/sec (drop-in get_images on NumPy windows, H2D included)",
        "value": world * n / step_s, "unit": "vehicle-pass windows/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic windows in host memory (NumPy float32)",
        "config": {"workload": "speeds-host", "baseline_config": wl["config"], "description": wl["desc"],
                   "windows_per_step": world * n, "window_mb": 4.0 * n_ch * n_t / 1e6,
                   "parallelism": f"dp{world} (replicas)"},
        "roofline": {"bound": "pcie", "achieved": win_bytes / step_s / 1e9, "peak": h2d, "unit": "GB/s",
                     "frac": win_bytes / step_s / 1e9 / h2d, "traffic": None,
                     "peak_source": "pinned 64 MB H2D copies measured in this run (PCIe Gen5 x16 spec 63 GB/s)",
                     "pcie_bound_windows_per_s": h2d * 1e9 / (4.0 * n_ch * n_t)},
        "avg_image_finite": bool(all(np.isfinite(x).all() for x in res_imgs)),
        "cpu_baseline": None,
    }
    # nothing in flight at exit: the staging side streams and the pinned table uploads are drained (under rocprofv3
    # the round-4 run ended with 26-30 asynchronous copies still unaccounted for)
    from das_diff_veh_amd.device import sync_staging
    sync_staging()
    torch.cuda.synchronize()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = _ARGS
    if args.pool:
        if "pool" not in WORKLOADS[args.workload]:
            raise SystemExit(f"[bench] --pool: workload {args.workload} has no window pool")
        WORKLOADS[args.workload]["pool"] = args.pool
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("DVH_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and local >= n_dev:
        # one rank per GPU: fewer visible GPUs than local ranks is a launch error, never two ranks on one device
        raise SystemExit(f"[bench] rank {rank}: LOCAL_RANK {local} but only {n_dev} visible GPU(s); RCCL runs one "
                         f"rank per GPU (DVH_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    if backend != "nccl":
        local %= max(1, n_dev)  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # RCCL over xGMI, one rank per GPU; DVH_DIST_BACKEND=gloo rehearses the multi-rank step with
        # several ranks on one GPU (RCCL refuses that), reducing through host copies
        # the collective libraries' own connection messages (Gloo prints one per rank on stdout) go to stderr:
        # stdout carries only rank 0's JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend, device_id=device if backend == "nccl" else None)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"[bench] world size {dist.get_world_size()} != --gpus {args.gpus}")

    kind = WORKLOADS[args.workload]["kind"]
    if kind in ("timelapse", "bootstrap", "prep", "host"):
        return {"timelapse": timelapse_main, "bootstrap": bootstrap_main, "prep": prep_main,
                "host": host_main}[kind](args, world, rank, device)
    if args.sliding_merge is not None:
        WORKLOADS["sliding"]["merge"] = args.sliding_merge
    if args.w499:
        if WORKLOADS[args.workload]["kind"] not in ("pool", "resident"):
            raise SystemExit("--w499 applies to synth10k / weights / speeds")
        WORKLOADS[args.workload]["t0"] = DT_W499
    scaling = args.scaling or ("weak" if world == 1 else "both")
    res = measure(args, "strong" if scaling == "strong" else "weak", world, rank, device,
                  cpu=rank == 0 and world == 1 and not args.no_cpu_baseline)
    if scaling == "both":
        # the fixed job of the configured size split over the ranks, measured beside the weak line
        strong = measure(args, "strong", world, rank, device, cpu=False)
        res["strong_scaling"] = {k: strong[k] for k in ("value", "ms_per_step", "scaling")}
        res["strong_scaling"].update({k: strong["config"][k] for k in ("windows_per_step", "windows_per_step_this_rank")})
        res["strong_scaling"]["stack_launch_ms"] = strong["roofline"]["launch_ms"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure(args, scaling, world, rank, device, cpu):
    """Build the workload's job for `scaling`, time args.steps steps after args.warmup, and return the
    result record (rank 0's view, elapsed = max over ranks)."""
    job = build(args.workload, device, world, rank, scaling, chunk=args.chunk)
    torch.cuda.synchronize()
    log(f"[bench] rank {rank}: {job.windows.shape[0]} resident windows generated in {job.t_gen:.2f}s, host setup "
        f"{job.t_plan:.2f}s; {job.n_local} passes per step on this rank ({job.units} units), "
        f"{len(job.batches)} batches, R = {job.batches[0].plan.R}")
    if args.layout_out and rank == 0:
        with open(args.layout_out, "w") as fh:
            json.dump(layout_of(job, args, scaling), fh)

    for _ in range(args.warmup):
        step(job, world, fused=not args.separate_validity)
    torch.cuda.synchronize()
    # algorithmic bytes of every stack launch (bookkeeping outside the timed region: a batch whose
    # tables share a buffer with others is re-derived first; each batch's tables are copied back once)
    fused = [bool(not args.separate_validity and b.validity and (b.plan.flags & 6)) for b in job.batches]
    corr_bytes, win_bytes = [], []
    out_bytes = 4 * job.stack.shape[0] * job.stack.shape[1] * job.stack.shape[2]
    for b in job.batches:
        if b.derive:
            b.plan.derive()
        corr_bytes.append(b.plan.algorithmic_bytes(out_rows=job.stack.shape[0] * job.stack.shape[1]))
        win_bytes.append(getattr(b, "scan_bytes", 4 * b.win.shape[0] * b.win.shape[1] * b.win.shape[2]) if b.validity
                         else 0)
    # a validated launch must read every window sample once (the correlation slices are subsets of
    # the window): its algorithmic bytes are the windows plus the stack rows written
    bytes_stack = [wb + out_bytes if f else cb for f, wb, cb in zip(fused, win_bytes, corr_bytes)]
    torch.cuda.synchronize()

    nb = len(job.batches)
    ev = [{p: [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(nb)]
           for p in PHASES} for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(job, world, ev[k], fused=not args.separate_validity)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, device)

    ms = {p: np.array([[ev[k][p][j][0].elapsed_time(ev[k][p][j][1]) for j in range(nb)] for k in range(args.steps)])
          for p in PHASES}
    windows_per_step = job.n_global
    images_per_step = job.stack.shape[0]
    # roofline of the dominant kernel (vsg_stack): algorithmic bytes per launch / mean launch time
    bytes_per_launch = float(np.mean(bytes_stack))
    launch_s = float(ms["stack"].mean()) / 1e3
    achieved = bytes_per_launch / launch_s / 1e9
    layout = layout_of(job, args, scaling)
    kname = "vsg_stackv_kernel" if all(fused) else "vsg_stackf_kernel"
    traffic, traffic_src = pmc_lookup(kname, layout, "traffic_bytes")
    step_ms = elapsed / args.steps * 1e3
    res = {
        "metric": "vehicle-pass windows/sec -> stacked VSG + f-v images/sec; % HBM/MFMA roofline",
        "value": windows_per_step * args.steps / elapsed,
        "unit": "vehicle-pass windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated dispersive moving-source wavefield, per-pass trajectories)",
        "config": {"workload": args.workload, "baseline_config": WORKLOADS[args.workload]["config"],
                   "description": WORKLOADS[args.workload]["desc"],
                   "windows_per_step": windows_per_step, "windows_per_step_this_rank": job.n_local,
                   "class_images_per_step": images_per_step, "gather_rows": job.batches[0].plan.R,
                   "w": job.batches[0].plan.w, "parallelism": f"dp{world} (passes sharded, all-reduce of class stacks)",
                   "chunk": args.chunk, "gather_units_per_step_this_rank": job.units, "stack_launches_per_step": nb},
        "images_per_s": images_per_step * args.steps / elapsed,
        "gather_units_per_s": job.units * (job.n_global / job.n_local) * args.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "vsg_stackv_kernel" if all(fused) else "vsg_stackf_kernel",
                     "bytes_per_launch": bytes_per_launch, "launch_ms": launch_s * 1e3,
                     "bytes_model": "every window sample once + stack rows written (validity read fused into the "
                                    "launch)" if all(fused) else "receiver samples under sub-windows + distinct pivot "
                                    "samples + stack rows written",
                     "correlation_bytes_per_launch": float(np.mean(corr_bytes)),
                     "correlation_frac": float(np.mean(corr_bytes)) / launch_s / 1e9 / HBM_PEAK_GBS},
        "step_breakdown_ms": {p: float(ms[p].sum(axis=1).mean()) for p in PHASES},
        "host_setup_s": job.t_plan,
    }
    res["step_breakdown_ms"]["fv_allreduce_rest"] = step_ms - sum(res["step_breakdown_ms"].values())
    if any(win_bytes) and not any(fused):
        vs = float(ms["validity"].mean()) / 1e3
        res["validity_roofline"] = {"kernel": "window_sumsq_kernel", "bytes_per_launch": float(np.mean(win_bytes)),
                                    "launch_ms": vs * 1e3, "achieved": float(np.mean(win_bytes)) / vs / 1e9,
                                    "frac": float(np.mean(win_bytes)) / vs / 1e9 / HBM_PEAK_GBS}
    valu, valu_src = pmc_lookup(kname, layout, "SQ_INSTS_VALU")
    res["valu_roofline"] = {"achieved": None if valu is None else valu / launch_s, "peak": VALU_PEAK_INSTR_S,
                            "unit": "wave-instr/s", "frac": None if valu is None else valu / launch_s / VALU_PEAK_INSTR_S,
                            "instr_per_launch": valu, "source": valu_src, "clock_assumed_ghz": 2.4,
                            "model": "wave64 VALU instruction = 2 cycles on a SIMD-32 (>= 2 waves per SIMD) at the "
                                     "2.4 GHz max clock"}
    if cpu and (job.cpu_sets or getattr(job, "cpu_units", None)):
        cb = cpu_baseline(job, args.cpu_budget) if job.cpu_sets else cpu_baseline_sliding(job, args.cpu_budget)
        res["cpu_baseline"] = cb
        res["speedup_vs_cpu"] = res["value"] / cb["value"]
    else:
        res["cpu_baseline"] = None
    del job
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    main()
