"""Stack-launch breakdown on one batch of a bench workload (default synth10k, BASELINE configs[2]), HIP-event timed:

    fused      vsg_stack_validated (correlation + whole-window scan in one launch, the bench's kernel)
    corr7      the same launch with a one-window scan: the correlation alone in the fused launch's layout
    corr       vsg_stack (the correlation alone, 4 waves per block)
    sumsq      window_sumsq of the batch (the validity as its own streaming pass)

    python tools/exp_stack.py [--reps 20] [--only fused,corr] [--workload synth10k|weights|speeds]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from das_diff_veh_amd.vsg import UnitScan, vsg_scales, vsg_stack, vsg_stack_validated, window_sumsq  # noqa: E402


def timed(fn, reps, stream):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    return float(np.median(ms)), float(ms.min())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="fused,corr7,corr,sumsq")
    ap.add_argument("--workload", default="synth10k", choices=("synth10k", "weights", "speeds"))
    ap.add_argument("--w499", action="store_true", help="time axes with w = 499 (zero-padded 1 024-point engine)")
    args = ap.parse_args()
    if args.w499:
        from das_diff_veh_amd.synth import DT_W499
        bench.WORKLOADS[args.workload]["t0"] = DT_W499
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    job = bench.build(args.workload, dev, 1, 0)
    b = job.batches[0]
    if getattr(job, "plan_all", None) is not None:
        job.plan_all.derive()
    elif b.derive:
        b.plan.derive()
    vsg_scales(b.win, b.plan, out=b.scales, win_sumsq=None, validity=False)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    n, C, T = b.win.shape
    one = UnitScan(np.zeros(1, np.int32), np.zeros(n, np.int32), C)
    # every pass's correlation reads pass 0's window (receivers hot in the caches), the scan still
    # reads every window: isolates what HBM latency under the scan costs the correlation
    assert b.win.stride(0) == C * b.win.stride(1)
    hot = b.win.as_strided((n, n * C, T), (0, b.win.stride(1), 1))  # rows span every window for the scan
    allw = UnitScan(np.arange(n, dtype=np.int32) * C, np.arange(n, dtype=np.int32), C)
    out = {}
    fns = {
        "fused": lambda: vsg_stack_validated(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, work=job.work),
        "corr7": lambda: vsg_stack_validated(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, work=job.work,
                                             scan=one),
        "fused_hot": lambda: vsg_stack_validated(hot, b.plan, b.sched, scales=b.scales, out=job.stack, work=job.work,
                                                 scan=allw),
        "corr7_hot": lambda: vsg_stack_validated(hot, b.plan, b.sched, scales=b.scales, out=job.stack, work=job.work,
                                                 scan=one),
        "corr_hot": lambda: vsg_stack(hot, b.plan, b.sched, scales=b.scales, out=job.stack),
        "corr": lambda: vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=job.stack),
        "sumsq": lambda: window_sumsq(b.win, out=b.sumsq),
    }
    for name in args.only.split(","):
        med, lo = timed(fns[name], args.reps, s)
        out[name] = dict(median_ms=round(med, 4), min_ms=round(lo, 4))
        print(name, out[name], file=sys.stderr, flush=True)
    out["n_pass"] = b.plan.n_pass
    out["corr_bytes"] = float(b.plan.algorithmic_bytes())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
