#!/usr/bin/env python
"""Throughput of the bootstrap / convergence path at notebook scale.

The notebooks' convergence_test (imaging_diff_speed.ipynb#cell30-31) runs bootstrap_disp for
bt_size = 1..60 with bt_times = 30 per class: 1,800 resampled class stacks, their f-v images and 4
ridge picks each (sigma / ref_freq_idx / bands / reference curves of #cell25).  This tool does one
class (mid-speed: 1,442 synthetic passes of 60 x 5,500) on one GPU and prints one JSON line:
resamples/s, the split between the one-off gathers and the resampling, and the reference's cost of
the same work on one host core from its measured per-window / per-image costs (bench.py's
cpu_baseline numbers, passed with --cpu-ms-window / --cpu-ms-image).

    python tools/bench_bootstrap.py [--n 1442] [--max-size 60] [--bt-times 30]
"""
import argparse
import json
import os
import random
import sys
import time
import types

import numpy as np
import scipy.interpolate
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from das_diff_veh_amd import bootstrap as bt  # noqa: E402
from das_diff_veh_amd.synth import synth_batch_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1442)
    ap.add_argument("--max-size", type=int, default=60)
    ap.add_argument("--bt-times", type=int, default=30)
    ap.add_argument("--cpu-ms-window", type=float, default=13.2)
    ap.add_argument("--cpu-ms-image", type=float, default=10.8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wins_t, x_axis, t_axis, trk, _ = synth_batch_device(args.n, pivot=700.0, seed=3, device=dev)
    wins = [types.SimpleNamespace(data=wins_t[i], x_axis=x_axis, t_axis=t_axis, veh_state_x=trk[i][0],
                                  veh_state_t=trk[i][1]) for i in range(args.n)]
    sigma = [25, 50, 50, 50]
    ref_idx = [80, 130, 170, 170]
    lb, ub = [2.5, 10, 14, 16], [14, 15, 19, 20]
    curves = [None,
              scipy.interpolate.interp1d([10, 12, 13, 14, 15, 16], [530, 470, 450, 430, 410, 391]),
              scipy.interpolate.interp1d([14, 15, 16, 17, 18, 19], [630, 583, 550, 520, 500, 490]),
              scipy.interpolate.interp1d([16, 17, 18, 19, 20, 21], [745, 690, 657, 626, 600, 580])]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cache = bt.GatherCache(wins, 700.0, 500.0, 900.0, device=dev)
    torch.cuda.synchronize()
    t_gather = time.perf_counter() - t0
    del wins_t
    # warm-up (plans, code objects)
    random.seed(0)
    bt.bootstrap_ridges(cache, bt.draw(args.n, 2, 2), sigma, ref_idx, lb, ub, curves)
    random.seed(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stds = np.empty((4, args.max_size))
    for k in range(1, args.max_size + 1):
        sels = bt.draw(args.n, k, args.bt_times)
        per_mode = bt.bootstrap_ridges(cache, sels, sigma, ref_idx, lb, ub, curves)
        for m, r in enumerate(per_mode):
            stds[m, k - 1] = np.sum(np.std(r, axis=0))
    torch.cuda.synchronize()
    t_resample = time.perf_counter() - t0
    n_res = args.max_size * args.bt_times
    windows_drawn = args.bt_times * args.max_size * (args.max_size + 1) // 2
    cpu_s = windows_drawn * args.cpu_ms_window / 1e3 + n_res * args.cpu_ms_image / 1e3
    print(json.dumps({
        "metric": "bootstrap resamples/s (convergence_test, one class)",
        "value": n_res / (t_gather + t_resample), "unit": "resamples/s", "n_gpus": 1,
        "config": {"passes": args.n, "bt_sizes": f"1..{args.max_size}", "bt_times": args.bt_times, "modes": 4,
                   "window": "60 x 5500", "disp_rows": "offsets -150..0 m"},
        "gathers_s": t_gather, "resampling_s": t_resample, "resamples": n_res,
        "cpu_reference_estimate_s": cpu_s, "cpu_basis": f"{windows_drawn} VSG gathers x {args.cpu_ms_window} ms + "
                                                        f"{n_res} f-v images x {args.cpu_ms_image} ms on 1 core "
                                                        "(bench.py cpu_baseline per-window / per-image costs), "
                                                        "ridge picks not counted",
        "speedup_vs_cpu_1core": cpu_s / (t_gather + t_resample),
        "std_sum_mode0_first_last": [float(stds[0, 0]), float(stds[0, -1])]}))


if __name__ == "__main__":
    main()
