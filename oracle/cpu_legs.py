"""All-core CPU-baseline workers (BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline legs run one of these per
usable host core, each a single-threaded process as the reference is).

    python -m oracle.cpu_legs KIND SAMPLE_DIR FIRST BUDGET_S   ->  one JSON line of counts and seconds

SAMPLE_DIR holds .npy arrays (memory-mapped, so the workers share one page-cache copy) and params.json.
Kinds, each the reference's own computation through the oracle restatements (pinned by tests/test_oracle.py):
  vsg   VirtualShotGather gathers (oracle/ref_loop.gather: the reference's per-row scipy.signal.correlate loop,
        apis/virtual_shot_gather.py:111-192 / modules/utils.py:253-314) of the saved windows round robin from FIRST
        until BUDGET_S, summed into a stack (apis/imaging_classes.py:106-107); then f-v images of the mean stack
        (ref_loop.disp_image: compute_disp_image -> map_fv, modules/utils.py:457-475) for up to a tenth of the budget
        (at least one) -> windows, secs, images, img_secs
  fv    map_fv of the saved gathers (configs[4]) -> images, secs
  prep  _preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71: scipy sosfiltfilt as bandpass_data calls
        it, the imputation quirks, the trace norm) of the saved record slice, repeated -> rows, secs
  boot  one bootstrap_disp resample's pieces (apis/imaging_classes.py:8-48): gathers for 70 % of the budget, then an
        f-v image of their mean (compute_disp_image(end_x=0, start_x=-150)) and the 4 ridge walks
        (extract_ridge_ref_idx, modules/utils.py:621-678) -> gathers, g_secs, img_secs, ridge_secs
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np


def _load(d):
    arr = {f[:-4]: np.load(os.path.join(d, f), mmap_mode="r", allow_pickle=False)
           for f in os.listdir(d) if f.endswith(".npy")}
    with open(os.path.join(d, "params.json")) as fh:
        return arr, json.load(fh)


def vsg(d, first, budget):
    from oracle import ref_loop
    a, p = _load(d)
    wins, vx, vt = a["wins"], a["vx"], a["vt"]
    n = wins.shape[0]
    piv, sx, ex = (np.broadcast_to(np.asarray(a[k] if k in a else p[k], dtype=np.float64), (n,))
                   for k in ("pivot", "start_x", "end_x"))
    acc, done, t0 = None, 0, time.perf_counter()
    while True:
        i = (first + done) % n
        g, gx, gt = ref_loop.gather(np.asarray(wins[i], np.float64), a["x_axis"], a["t_axis"], vx[i], vt[i], piv[i],
                                    sx[i], ex[i])
        acc = g if acc is None else acc + g
        done += 1
        secs = time.perf_counter() - t0
        if secs >= budget:
            break
    m, n_img, t1 = acc / done, 0, time.perf_counter()
    while True:
        ref_loop.disp_image(m, gx, gt, start_x=p.get("disp_start_x", -200), end_x=p.get("disp_end_x", 0))
        n_img += 1
        img = time.perf_counter() - t1
        if img >= budget / 10:
            break
    return dict(windows=done, secs=secs, images=n_img, img_secs=img)


def fv(d, first, budget):
    from oracle import disp as odisp
    a, p = _load(d)
    g = a["gathers"]
    freqs, vels = np.asarray(a["freqs"]), np.asarray(a["vels"])
    done, t0 = 0, time.perf_counter()
    while True:
        odisp.map_fv(np.asarray(g[(first + done) % g.shape[0]], np.float64), p["dx"], p["dt"], freqs, vels)
        done += 1
        secs = time.perf_counter() - t0
        if secs >= budget:
            return dict(images=done, secs=secs)


def prep(d, first, budget):
    from oracle import preprocess as oprep
    a, p = _load(d)
    rec = np.asarray(a["record"])
    done, t0 = 0, time.perf_counter()
    while True:
        oprep.surface_wave_prep(rec, p["dt"], scipy_filter=True)
        done += 1
        secs = time.perf_counter() - t0
        if secs >= budget:
            return dict(rows=done * rec.shape[0], secs=secs)


def boot(d, first, budget):
    import scipy.interpolate

    from oracle import ref_loop
    from oracle import ridge as orid
    a, p = _load(d)
    wins, vx, vt = a["wins"], a["vx"], a["vt"]
    n = wins.shape[0]
    gs, t0 = [], time.perf_counter()
    while True:
        i = (first + len(gs)) % n
        g, gx, gt = ref_loop.gather(np.asarray(wins[i], np.float64), a["x_axis"], a["t_axis"], vx[i], vt[i], p["pivot"],
                                    p["start_x"], p["end_x"])
        gs.append(g)
        g_secs = time.perf_counter() - t0
        if g_secs >= 0.7 * budget:
            break
    t1 = time.perf_counter()
    fvm = ref_loop.disp_image(np.mean(gs, axis=0), gx, gt, start_x=-150, end_x=0)
    img = time.perf_counter() - t1
    fq, vels = np.arange(0.8, 25, 0.1), np.arange(200, 1200)
    curves = [None if c is None else scipy.interpolate.interp1d(*c) for c in p["curves"]]
    t2 = time.perf_counter()
    for m in range(len(p["sigma"])):
        band = (fq >= p["lb"][m]) & (fq < p["ub"][m])
        try:
            orid.extract_ridge_ref_idx(fq[band], vels, fvm[:, band], ref_freq_idx=p["ref_idx"][m] - int(np.sum(fq < p["lb"][m])),
                                       sigma=p["sigma"][m], vel_max=800, ref_vel=curves[m])
        except ValueError:
            pass
    return dict(gathers=len(gs), g_secs=g_secs, img_secs=img, ridge_secs=time.perf_counter() - t2)


if __name__ == "__main__":
    kind, sample, first, budget = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
    print(json.dumps({"vsg": vsg, "fv": fv, "prep": prep, "boot": boot}[kind](sample, first, budget)), flush=True)
