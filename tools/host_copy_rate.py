"""Host-side rates behind the host-fed bench (bench.py --workload speeds-host): the packing copy of NumPy windows
into pinned memory (device.stage_windows' host half, dvh_host_gather on N threads and np.copyto), alone, and the
pinned H2D copy alone.  Prints one JSON line.

    python tools/host_copy_rate.py [--windows 2108] [--threads 16]
"""
import argparse
import concurrent.futures as cf
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from das_diff_veh_amd import _lib  # noqa: E402
from das_diff_veh_amd.device import STAGE_BYTES  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=2108)
ap.add_argument("--threads", type=int, default=16)
args = ap.parse_args()

rng = np.random.default_rng(0)
hosts = [rng.standard_normal((60, 5500), dtype=np.float32) for _ in range(args.windows)]
per = hosts[0].nbytes
k = STAGE_BYTES // per
pinned = torch.empty(k * per, dtype=torch.uint8, pin_memory=True)
base = pinned.data_ptr()
view = pinned.numpy().view(np.float32).reshape(k, 60, 5500)
out = {"windows": args.windows, "window_mb": per / 1e6, "chunk_windows": k}


def run(mode, nt):
    pool = cf.ThreadPoolExecutor(nt)
    t0 = time.perf_counter()
    for a in range(0, len(hosts), k):
        chunk = hosts[a:a + k]
        kk = len(chunk)
        n = min(kk, nt)
        bounds = [kk * q // n for q in range(n + 1)]
        srcs = (ctypes.c_void_p * kk)(*[h.ctypes.data for h in chunk])
        if mode == "native":
            def f(q):
                j0, j1 = bounds[q], bounds[q + 1]
                _lib.call("dvh_host_gather", ctypes.c_void_p(base + j0 * per),
                          ctypes.byref(srcs, j0 * ctypes.sizeof(ctypes.c_void_p)), per, j1 - j0)
        else:
            def f(q):
                for j in range(bounds[q], bounds[q + 1]):
                    np.copyto(view[j], chunk[j])
        list(pool.map(f, range(n)))
    dt = time.perf_counter() - t0
    pool.shutdown()
    return len(hosts) * per / dt / 1e9


for mode in ("native", "numpy"):
    for nt in (8, args.threads, 2 * args.threads):
        run(mode, nt)  # warm
        out[f"{mode}_{nt}t_GBs"] = round(max(run(mode, nt) for _ in range(2)), 2)
dev = torch.empty(k * per, dtype=torch.uint8, device="cuda")
dev.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    dev.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
out["h2d_pinned_GBs"] = round(10 * k * per / (time.perf_counter() - t0) / 1e9, 2)
print(json.dumps(out))
