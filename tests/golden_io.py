"""Loading helpers for the golden fixtures in tests/golden/ (written by make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
QUANT = 2.0 ** -12


def load(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)


def n_pass(g, prefix=""):
    return g[prefix + "q"].shape[0]


def pass_arrays(g, i, prefix=""):
    """Constructor arguments of a SurfaceWaveWindow for pass i of a fixture."""
    return dict(data=g[prefix + "q"][i].astype(np.float32) * np.float32(QUANT),
                x_axis=g[prefix + "x_axis"][i], t_axis=g[prefix + "t_axis"][i],
                veh_state=g[prefix + "veh_state"][i], start_x_tracking=float(g[prefix + "start_x_tracking"][i]),
                distance_along_fiber_tracking=g[prefix + "distance_along_fiber_tracking"],
                t_axis_tracking=g[prefix + "t_axis_tracking"][i])


def oracle_window(g, i, prefix=""):
    from oracle import vsg
    a = pass_arrays(g, i, prefix)
    vx, vt = vsg.veh_state_xt(a["veh_state"], a["start_x_tracking"], a["distance_along_fiber_tracking"],
                              a["t_axis_tracking"])
    return dict(data=a["data"].astype(np.float64), x_axis=a["x_axis"], t_axis=a["t_axis"], veh_state_x=vx,
                veh_state_t=vt)


def gather_rel_err(got, ref):
    """max |got - ref| / max |ref| over the finite reference entries; NaN/inf positions must agree."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    assert np.array_equal(np.isposinf(got), np.isposinf(ref)), "+inf pattern differs"
    assert np.array_equal(np.isneginf(got), np.isneginf(ref)), "-inf pattern differs"
    m = np.isfinite(ref)
    if not m.any():
        return 0.0
    scale = np.abs(ref[m]).max()
    return float(np.abs(got[m] - ref[m]).max() / (scale if scale > 0 else 1.0))


def select_cases():
    """Synthetic continuous records + tracked vehicles for SurfaceWaveSelector.locate_windows
    (apis/data_classes.py:170-223).  veh_states holds tracking-time indices per tracking channel
    (NaN off the tracked span); x0 - start_x_tracking indexes its column, as the reference does."""
    rng = np.random.default_rng(700)
    n_ch, n_t, dt = 48, 6000, 0.004
    dist = 400.0 + 8.16 * np.arange(n_ch)             # distances_along_fiber of the record
    dist_trk = 380.0 + 4.08 * np.arange(160)          # tracking grid (finer, offset)
    t_trk = np.arange(0, n_t * dt, 0.012)             # tracking time axis (3 record samples)
    rec = np.round(rng.standard_normal((n_ch, n_t)) * 2 ** 8) / 2 ** 8  # exact in float32
    n_x = 60

    def states(tc):
        """tracking-time indices of vehicles crossing column 25 at times tc (0.05 s per column)"""
        vs = np.full((len(tc), n_x), np.nan)
        for k, t in enumerate(tc):
            times = t + (np.arange(n_x) - 25) * 0.05
            ok = (times >= 0) & (times < t_trk[-1])
            vs[k, ok] = np.round(times[ok] / 0.012)
            vs[k, :3] = np.nan                         # untracked head of the span
        return vs

    base = dict(rec=rec, dist=dist, t_axis=np.arange(n_t) * dt, x0=620, start_x_tracking=595, dist_trk=dist_trk,
                t_trk=t_trk)
    # crossing times at column x0_idx = 25, in pass order: spacings exercise car-behind (< spacing to the
    # next), car-ahead (0 <= delta < spacing), a negative delta (not "ahead") and both record boundaries
    mixed = [0.5, 3.0, 4.0, 4.9, 6.0, 9.9, 10.0, 7.0, 11.7, 14.0, 18.5, 20.2, 23.004]
    return {
        "default": dict(base, veh_states=states([3.0, 5.0, 13.5, 22.0, 23.5]), kw={}),  # 2000-sample windows
        "short": dict(base, veh_states=states(mixed), kw=dict(wlen_sw=2, length_sw=120, spatial_ratio=0.5)),
        # 499-sample windows: the last crossing sits where t0 + 249 == n_t, so its slice is clipped to 498
        "odd": dict(base, veh_states=states(mixed), kw=dict(wlen_sw=1.998, length_sw=100, spatial_ratio=0.25,
                                                              temporal_spacing=0.5)),
        "spacing": dict(base, veh_states=states(mixed), kw=dict(wlen_sw=1, length_sw=150, temporal_spacing=1.05)),
    }


def workflow_files():
    """Two synthetic "files" of one day for ImagingWorkflowOneDirectory.imaging (apis/imaging_workflow.py:33-80)
    with method='xcorr': continuous records of 48 ch x 9 000 samples on a time axis starting at t = 4 s (so that no
    window's t_axis[1] - t_axis[0] is exactly 0.004, where the reference raises; the windows' steps then round to
    w = 500 or 499 by their start, and the class means mix both, as on real records), tracked vehicles at varied
    speeds (seconds per 1 m tracking column), x0 = 620; wlen_sw = 12 s windows (3 000 samples: room for the pivot's
    4 s correlation window on both sides).  File A accepts 2 of 3 passes (the last window runs past the record),
    file B 2 of 3 (the same)."""
    from das_diff_veh_amd.synth import DT_W500
    n_ch, n_t, dt = 48, 9000, 0.004
    dist_trk = 380.0 + np.arange(400.0)  # the 1 m tracking grid (resample_poly 204 / 25 of the 8.16 m channels)
    t_trk = DT_W500 + np.arange(0, n_t * dt, 0.012)
    n_x = 100

    def states(tc, spc):
        vs = np.full((len(tc), n_x), np.nan)
        for k, (t, s) in enumerate(zip(tc, spc)):
            times = t + (np.arange(n_x) - 25) * s
            ok = (times >= 0) & (times < t_trk[-1])
            vs[k, ok] = np.round(times[ok] / 0.012)
            vs[k, :2] = np.nan
        return vs

    files = []
    for seed, tc, spc in ((710, [7.0, 19.5, 32.0], [0.05, 0.04, 0.06]), (711, [6.2, 18.4, 30.6], [0.055, 0.045, 0.05])):
        rng = np.random.default_rng(seed)
        rec = np.round(rng.standard_normal((n_ch, n_t)) * 2 ** 8) / 2 ** 8  # exact in float32
        files.append(dict(rec=rec, x_axis=449.0 + np.arange(n_ch), t_axis=DT_W500 + np.arange(n_t) * dt, x0=620,
                          start_x_tracking=595, veh_states=states(tc, spc), dist_trk=dist_trk, t_trk=t_trk,
                          select_kw=dict(wlen_sw=12, length_sw=300, spatial_ratio=0.75),
                          imaging_kw=dict(pivot=620, start_x=500, end_x=680, wlen=2, include_other_side=True)))
    return files
