#!/usr/bin/env python
"""BASELINE configs[4] (time-lapse): batched f-v images of daily class stacks on one MI355X.

One step = the f-v images of B gathers (one day's stacks at B pivots, the [-200, 0] m rows of a
49 x 500 gather: 25 channels x 500 lags) on a 512-velocity x 1,000-frequency grid (compute_disp_image
-> Dispersion -> map_fv, modules/utils.py:383-426, 457-475), through the dispersion kernels:
  tdft_*_kernel       time DFT as a real float64 MFMA GEMM [B*nch x nt] . [nt x 2*n_fb] (tdft_rows_kernel:
                      LDS-staged twiddles; the key "tdft_gemm_kernel" below is the time-DFT launch, either kernel)
  fk_contract_kernel  channel contraction, complex float64 MFMA GEMM per gather, |.|
  fv_*_kernel         FITPACK bilinear sampling + Savitzky-Golay(25, 4), float32 out (the product dispatch:
                      fv_mfma_kernel, the filter as banded float64 MFMA GEMMs, for a batch this size)
Per-kernel durations come from HIP events on the launch stream; the GEMM rooflines are priced
against the float64 MFMA peak, fv_kernel against HBM (it writes 4 * nV * nF bytes per image).
The gathers are synthetic (dispersive tones c(f) = 250 + 4000 / (f + 4), noise), resident on the
device before timing; two images are checked against the oracle (oracle/disp.py) after timing.

    python tools/bench_timelapse.py [--batch 512] [--steps 10] [--warmup 2] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from das_diff_veh_amd import _lib  # noqa: E402
from das_diff_veh_amd.disp import DispPlan, fv_from_fk  # noqa: E402
from das_diff_veh_amd.synth import synth_gathers  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip parameters
FP64_MFMA_PEAK_TF = 47.8       # v_mfma_f64_16x16x4_f64 measured on the box (tools/calib/dp_pipes); spec sheet 78.6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nv", type=int, default=512)
    ap.add_argument("--nf", type=int, default=1000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nch, nt, dx, dt = 25, 500, 8.16, 0.003999999999997783
    freqs = np.linspace(1.0, 25.0, args.nf)
    vels = np.linspace(200.0, 1200.0, args.nv)
    plan = DispPlan(nch, nt, dx, dt, freqs, vels)
    B = args.batch
    data = synth_gathers(B, nch, nt, dx, dt, dev)
    tb = plan.tables(dev)
    st = _lib.stream_of(dev)
    D = torch.empty((B * nch, 2 * plan.n_fb), dtype=torch.float64, device=dev)
    FK = torch.empty((B, plan.n_kb, plan.n_fb), dtype=torch.float64, device=dev)
    fv = torch.empty((B, plan.nV, plan.nF), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

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
        fv_from_fk(FK, plan, out=fv)  # the product dispatch (cell-staged tiles for a batch this size)
        if ev:
            ev[3].record(stream)

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    for k in range(args.steps):
        run(evs[k])
    torch.cuda.synchronize()
    t = np.array([[e[i].elapsed_time(e[i + 1]) for i in range(3)] for e in evs]).mean(axis=0) / 1e3  # s
    step = float(np.array([e[0].elapsed_time(e[3]) for e in evs]).mean()) / 1e3

    # parity: two images against the oracle (float64 reference path)
    from oracle import disp as odisp
    host = data.double().cpu().numpy()
    errs, picks = [], []
    for b in (0, B - 1):
        ref = odisp.map_fv(host[b], dx, dt, freqs, vels)
        got = fv[b].double().cpu().numpy()
        errs.append(float(np.abs(got - ref).max() / np.abs(ref).max()))
        picks.append(bool(np.all(odisp.pick_ok(ref, got.argmax(axis=0)))))

    M, K, N = B * nch, nt, 2 * plan.n_fb
    tdft_flop = 2.0 * M * K * N
    fk_flop = 2.0 * B * (2 * plan.MT) * plan.K2 * plan.n_fb
    fv_bytes = 4.0 * B * plan.nV * plan.nF + 8.0 * B * plan.n_kb * plan.n_fb
    from das_diff_veh_amd.disp import _use_mfma
    mfma = _use_mfma(plan, B)
    fir_flop = 2.0 * 25 * B * plan.nV * plan.nF
    n_tiles = -(-(plan.nF - 16) // 16) + 1
    mfma_flop = 2.0 * 16 * 16 * 40 * n_tiles * B * -(-plan.nV // 16)
    res = {
        "metric": "time-lapse f-v images/s (configs[4]: 512 velocities x 1,000 frequencies, batched MFMA dispersion)",
        "value": B / step, "unit": "f-v images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step * 1e3, "dtype": "f64 MFMA (DFT / contraction), f32 out",
        "data": "synthetic dispersive gathers, resident", "config": {
            "workload": "timelapse", "gathers_per_step": B, "nch": nch, "nt": nt, "nV": plan.nV, "nF": plan.nF,
            "n_fb": plan.n_fb, "n_kb": plan.n_kb, "nf": plan.nf, "nk": plan.nk},
        "kernels": {
            "tdft_gemm_kernel": {"us": t[0] * 1e6, "flop": tdft_flop, "achieved_tflops": tdft_flop / t[0] / 1e12,
                                 "peak_tflops": FP64_MFMA_PEAK_TF, "frac": tdft_flop / t[0] / 1e12 / FP64_MFMA_PEAK_TF},
            "fk_contract_kernel": {"us": t[1] * 1e6, "flop": fk_flop, "achieved_tflops": fk_flop / t[1] / 1e12,
                                   "peak_tflops": FP64_MFMA_PEAK_TF, "frac": fk_flop / t[1] / 1e12 / FP64_MFMA_PEAK_TF},
            "fv_kernel": {"us": t[2] * 1e6, "bytes": fv_bytes, "achieved_gbs": fv_bytes / t[2] / 1e9,
                          "peak_gbs": HBM_PEAK_GBS, "frac": fv_bytes / t[2] / 1e9 / HBM_PEAK_GBS,
                          "kernel": "fv_mfma_kernel" if mfma else "fv_tile_kernel / fv_batch_kernel / fv_kernel",
                          # the Savitzky-Golay FIR (25 taps per output) and, for the MFMA kernel, the FLOPs it issues
                          # (10 v_mfma_f64_16x16x4_f64 per 16 x 16 tile, ceil((nF - 16) / 16) + 1 tiles per row)
                          "fir_flop": fir_flop, "mfma_flop_issued": mfma_flop if mfma else 0.0,
                          "mfma_frac": (mfma_flop / t[2] / 1e12 / FP64_MFMA_PEAK_TF) if mfma else None},
        },
        "parity": {"max_rel_err": max(errs), "picks_ok": all(picks), "images_checked": 2, "tol": 1e-4},
    }
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
