"""Experiment: does window_sumsq (HBM-bound) overlap with vsg_stack (VALU-bound) on two streams?"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import bench
from das_diff_veh_amd.vsg import vsg_scales, vsg_stack, window_sumsq

dev = torch.device("cuda:0")
job = bench.build("synth10k", dev, 1, 0, "weak", chunk=8)
b = job.batches[0]
b.plan.derive()
window_sumsq(b.win, out=b.sumsq)
vsg_scales(b.win, b.plan, out=b.scales, win_sumsq=b.sumsq)
torch.cuda.synchronize()
s2 = torch.cuda.Stream()
sumsq2 = torch.empty_like(b.sumsq)

def t(fn, n=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3

stack = lambda: vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=True)
val = lambda: window_sumsq(b.win, out=sumsq2)
def both():
    ev = torch.cuda.Event(); ev.record()
    with torch.cuda.stream(s2):
        s2.wait_event(ev)
        window_sumsq(b.win, out=sumsq2)
    vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=True)
    torch.cuda.current_stream().wait_stream(s2)
def both_rev():
    ev = torch.cuda.Event(); ev.record()
    vsg_stack(b.win, b.plan, b.sched, scales=b.scales, out=job.stack, accumulate=True)
    with torch.cuda.stream(s2):
        s2.wait_event(ev)
        window_sumsq(b.win, out=sumsq2)
    torch.cuda.current_stream().wait_stream(s2)
print("stack ms", t(stack), "validity ms", t(val), "both(val first) ms", t(both), "both(stack first) ms", t(both_rev), flush=True)
