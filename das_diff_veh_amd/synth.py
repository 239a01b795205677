"""Synthetic vehicle-pass DAS windows (the reference's pickled windows are not in the repo).

The reference's notebooks load ``data/sw_data/{600,700}.pkl`` (``imaging_diff_speed.ipynb#cell2``),
which are absent.  This module builds stand-ins with the same structure as a
``SurfaceWaveWindow`` (``apis/data_classes.py:12-39``): a channel-major ``data [C, T]`` block, a
channel axis in metres (8.16 m spacing), a time axis, and a vehicle trajectory expressed in the
tracking grid (1 m in distance, 50 Hz in time) exactly as ``KF_tracking`` emits it.

Wavefield model: a vehicle moving at constant speed radiates a dispersive
surface wave with phase velocity ``c(f) = 250 + 4000 / (f + 4)`` m/s and amplitude
``1 / (1 + d / 50)`` at distance ``d`` from the car, plus a quasi-static depression under the
car and white noise.  Samples are quantised to multiples of ``2**-12`` so that a window is
exactly representable both as fp32 (the device dtype) and as int16 (the fixture storage).
"""
from __future__ import annotations

import numpy as np

QUANT = 2.0 ** -12
DT_W500 = 4.0  # t0 for which (t0 + 0.004) - t0 == 0.0039999999999995595  -> w = 500, nsamp = 1000
DT_W499 = 30.0  # t0 for which the difference is 0.004000000000001336     -> w = 499, nsamp = 999
TRACK_DT = 0.02  # 50 Hz tracking grid (apis/timeLapseImaging.py:88)


def phase_velocity(f):
    return 250.0 + 4000.0 / (f + 4.0)


def synth_pass(seed, n_ch=56, n_t=4096, dx=8.16, x_first=472.0, t0=DT_W500, dt=0.004,
               pivot=700.0, speed=None, n_tones=24, noise=0.05, tc_offset=None,
               start_x_tracking=350.0, track_len=700, nan_head=5, nan_tail=5):
    """One synthetic pass as a dict of the arrays a ``SurfaceWaveWindow`` is built from."""
    rng = np.random.default_rng(seed)
    if speed is None:
        speed = float(rng.uniform(15.0, 30.0))
    if tc_offset is None:
        tc_offset = float(rng.uniform(-1.0, 1.0))
    x_axis = x_first + dx * np.arange(n_ch)
    t_axis = t0 + np.arange(n_t) * dt
    tc = t_axis[n_t // 2] + tc_offset  # time the car crosses the pivot

    # Tracking grid: 1 m distance axis, 50 Hz time axis on the same clock as t_axis.
    dist_trk = np.arange(0.0, 1600.0)
    t_trk = (t0 - 30.0) + np.arange(int((n_t * dt + 60.0) / TRACK_DT)) * TRACK_DT
    i0 = int(np.abs(start_x_tracking - dist_trk).argmin())
    xs = dist_trk[i0:i0 + track_len]
    t_at_x = tc + (xs - pivot) / speed
    idx = np.round((t_at_x - t_trk[0]) / TRACK_DT)
    veh_state = idx.astype(np.float64)
    veh_state[(idx < 0) | (idx >= t_trk.size)] = np.nan
    veh_state[:nan_head] = np.nan
    if nan_tail:
        veh_state[-nan_tail:] = np.nan

    xc = pivot + speed * (t_axis - tc)
    d = np.abs(x_axis[:, None] - xc[None, :])
    amp = 1.0 / (1.0 + d / 50.0)
    freqs = rng.uniform(2.0, 25.0, n_tones)
    phases = rng.uniform(0.0, 2.0 * np.pi, n_tones)
    u = np.zeros((n_ch, n_t))
    for f, ph in zip(freqs, phases):
        u += np.cos(2.0 * np.pi * f * (t_axis[None, :] - d / phase_velocity(f)) + ph)
    u *= amp * (2.0 / np.sqrt(n_tones))
    u -= 1.5 * np.exp(-(d / 15.0) ** 2)
    u += noise * rng.standard_normal((n_ch, n_t))
    q = np.clip(np.round(u / QUANT), -32767, 32767).astype(np.int16)
    return dict(q=q, data=q.astype(np.float32) * np.float32(QUANT), x_axis=x_axis, t_axis=t_axis,
                veh_state=veh_state, start_x_tracking=float(start_x_tracking),
                distance_along_fiber_tracking=dist_trk, t_axis_tracking=t_trk,
                speed=speed, tc=tc)


def linear_trajectory(x_axis_track, speed, tc, pivot):
    """(veh_state_x, veh_state_t) of a constant-speed pass, for batched synthetic workloads."""
    return x_axis_track, tc + (x_axis_track - pivot) / speed


def synth_batch_device(n_pass, n_ch=60, n_t=5500, dx=8.16, x_first=None, t0=DT_W500, dt=0.004, pivot=700.0,
                       seed=0, device="cuda", n_tones=8, noise=0.05, chunk=64, track_half=350, out=None):
    """A batch of synthetic passes generated on the device (same wavefield model as synth_pass,
    fewer tones), for throughput runs.  Returns (windows [n, C, T] float32, x_axis, t_axis,
    per-pass tracked trajectories (veh_state_x, veh_state_t) on the 1 m / 50 Hz tracking grid,
    speeds).  ``out`` (optional) is a caller-owned [n, C, T] float32 buffer (e.g. a slice of one
    resident buffer holding several window sets) written in place."""
    import torch
    rng = np.random.default_rng(seed)
    if x_first is None:
        x_first = pivot - 30 * dx + 0.37
    x_axis = x_first + dx * np.arange(n_ch)
    t_axis = t0 + np.arange(n_t) * dt
    speeds = rng.uniform(15.0, 30.0, n_pass)
    tcs = t_axis[n_t // 2] + rng.uniform(-1.0, 1.0, n_pass)
    freqs = rng.uniform(2.0, 25.0, n_tones)
    phases = rng.uniform(0.0, 2.0 * np.pi, (n_pass, n_tones))
    if out is None:
        out = torch.empty((n_pass, n_ch, n_t), dtype=torch.float32, device=device)
    elif tuple(out.shape) != (n_pass, n_ch, n_t) or out.dtype != torch.float32:
        raise ValueError("out must be a float32 [n_pass, n_ch, n_t] tensor")
    gen = torch.Generator(device=device)
    gen.manual_seed(int(seed) + 12345)
    xs = torch.as_tensor(x_axis, dtype=torch.float32, device=device)[None, :, None]
    for b in range(0, n_pass, chunk):
        e = min(b + chunk, n_pass)
        n = e - b
        trel = torch.as_tensor(t_axis[None, :] - tcs[b:e, None], dtype=torch.float32, device=device)  # [n, T]
        v = torch.as_tensor(speeds[b:e], dtype=torch.float32, device=device)[:, None]
        xc = (pivot + v * trel)[:, None, :]                       # [n, 1, T]
        d = (xs - xc).abs()                                      # [n, C, T]
        amp = 1.0 / (1.0 + d / 50.0)
        u = torch.zeros((n, n_ch, n_t), dtype=torch.float32, device=device)
        ph = torch.as_tensor(phases[b:e], dtype=torch.float32, device=device)
        for j, f in enumerate(freqs):
            c = float(phase_velocity(f))
            u += torch.cos(2.0 * np.pi * f * (trel[:, None, :] - d / c) + ph[:, j, None, None])
        u *= amp * (2.0 / np.sqrt(n_tones))
        u -= 1.5 * torch.exp(-(d / 15.0) ** 2)
        u += noise * torch.randn((n, n_ch, n_t), generator=gen, dtype=torch.float32, device=device)
        out[b:e] = torch.round(u / QUANT) * QUANT
    xs_trk = np.arange(np.floor(pivot) - track_half, np.floor(pivot) + track_half + 1, 1.0)
    trk = []
    for v, tc in zip(speeds, tcs):
        t = tc + (xs_trk - pivot) / v
        trk.append((xs_trk, np.round(t / TRACK_DT) * TRACK_DT))
    return out, x_axis, t_axis, trk, speeds


def synth_gathers(B, nch, nt, dx, dt, device, seed=0):
    """B gather-shaped [nch, nt] float32 blocks on the device (offsets 0, -dx, ...; lags centred):
    12 dispersive tones c(f) with random phases under a 0.6 s Gaussian lag envelope, plus noise --
    stand-ins for class-stack gathers in dispersion throughput and parity runs."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = -dx * torch.arange(nch, device=device, dtype=torch.float64)[:, None]
    t = (torch.arange(nt, device=device, dtype=torch.float64) - nt // 2)[None, :] * dt
    out = torch.zeros((B, nch, nt), dtype=torch.float64, device=device)
    rng = np.random.default_rng(seed)
    for f in rng.uniform(2.0, 24.0, 12):
        ph = torch.rand((B, 1, 1), generator=g, device=device, dtype=torch.float64) * 2 * np.pi
        out += torch.cos(2 * np.pi * f * (t + x / phase_velocity(f)) + ph) * torch.exp(-(t / 0.6) ** 2)
    out += 0.05 * torch.randn((B, nch, nt), generator=g, device=device, dtype=torch.float64)
    return out.float().contiguous()
