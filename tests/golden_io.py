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
