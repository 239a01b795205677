"""Host-side timeline of the host-fed step (bench.py --workload speeds-host: three classes' get_images on NumPy
windows): when each class's call starts, its windows' grouping and tables are done, its staged batch is waited
for, its stack launch is issued and the call returns, plus the span of its packing copies (dvh_host_gather, on
the staging threads).  Times in ms from the step's start, one warm step.

    python tools/host_timeline.py
"""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from das_diff_veh_amd import _lib, engine  # noqa: E402
from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow  # noqa: E402
from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows  # noqa: E402
from das_diff_veh_amd.synth import synth_batch_device  # noqa: E402

EV = []
lock = threading.Lock()


def mark(name):
    with lock:
        EV.append((time.perf_counter(), name, threading.get_ident()))


def wrap(mod, attr, name):
    fn = getattr(mod, attr)

    def w(*a, **k):
        mark(name + ">")
        r = fn(*a, **k)
        mark(name + "<")
        return r
    setattr(mod, attr, w)


wrap(engine, "_groups", "groups")
wrap(engine, "_plan", "plan")
wrap(engine, "vsg_stack_validated", "launch")
wrap(engine, "vsg_stack", "launch")
wrap(VirtualShotGathersFromWindows, "get_images", "get_images")
wrap(engine, "pack_trajectories_checked", "  pack")
wrap(engine, "_shared_or_stacked", "  axes")
wrap(engine.DevicePlan, "__init__", "  plan_init")
wrap(engine.DevicePlan, "derive", "  derive")
wrap(engine.DevicePlan, "check", "  check")
_call = _lib.call


def call(name, *a):
    if name != "dvh_host_gather":
        return _call(name, *a)
    mark("copy>")
    r = _call(name, *a)
    mark("copy<")
    return r


_lib.call = call
_rows = engine._rows_of


def rows_of(*a):
    f = _rows(*a)

    def g():
        mark("wait>")
        r = f()
        mark("wait<")
        return r
    return g


engine._rows_of = rows_of

dev = torch.device("cuda", 0)
n = 2108
w_dev, x_axis, t_axis, trk, _ = synth_batch_device(n, pivot=700.0, seed=5, device=dev)
host = w_dev.cpu().numpy()
del w_dev
wins = []
for i in range(n):
    w = SurfaceWaveWindow.__new__(SurfaceWaveWindow)
    w.data, w.x_axis, w.t_axis = np.ascontiguousarray(host[i]), x_axis, t_axis
    w.veh_state_x, w.veh_state_t = trk[i]
    wins.append(w)
cls = np.repeat(np.arange(3), (330, 1442, 336))
per = [[wins[i] for i in np.flatnonzero(cls == c)] for c in range(3)]
kw = dict(include_other_side=True, pivot=700, start_x=500, end_x=900, wlen=2)


def step():
    for ws in per:
        im = VirtualShotGathersFromWindows(ws)
        im.get_images(**kw)
        _ = im.avg_image.XCF_out


step()
torch.cuda.synchronize()
EV.clear()
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
t1 = time.perf_counter()
print(f"step {1e3 * (t1 - t0):.1f} ms")
main = threading.get_ident()
cls_i, copy_first, copy_last = -1, None, None
for t, name, tid in EV:
    ms = 1e3 * (t - t0)
    if name == "get_images>":
        cls_i += 1
        copy_first = copy_last = None
    if name.startswith("copy"):
        copy_first = ms if copy_first is None else copy_first
        copy_last = ms
        continue
    extra = ""
    if name == "get_images<" and copy_first is not None:
        extra = f"   (packing copies {copy_first:.2f} .. {copy_last:.2f})"
    print(f"class {cls_i}  {ms:8.2f}  {name}{extra}")
