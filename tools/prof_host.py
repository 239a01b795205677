"""Host-side profile of the drop-in get_images on NumPy windows (bench.py --workload speeds-host's step):
cProfile of one warm step, top functions by cumulative time.

    python tools/prof_host.py
"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow  # noqa: E402
from das_diff_veh_amd.apis.imaging_classes import VirtualShotGathersFromWindows  # noqa: E402
from das_diff_veh_amd.synth import synth_batch_device  # noqa: E402

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
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
print(f"step {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
