"""GPU parity of window selection: SurfaceWaveSelector (apis/data_classes.py:
126-223) against the reference's windows (tests/golden/select.npz): the accepted passes, the cut data
(bit-exact copies, dvh_cut_windows), the axes and the tracked trajectory samples of every window."""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
CASES = ["default", "short", "odd", "spacing"]


def _select(c, data):
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveSelector
    return SurfaceWaveSelector(data, c["dist"], c["t_axis"], c["x0"], c["start_x_tracking"], c["veh_states"],
                               c["dist_trk"], c["t_trk"], **c["kw"])


def _check(sel, c, g, case, to_host):
    ref = g[case + "_windows"]
    assert len(sel) == ref.shape[0]
    for w, (k, sx, ex, st, et) in zip(sel.windows, ref.tolist()):
        d = to_host(w.data)
        assert np.array_equal(d, c["rec"][sx:ex, st:et]), case
        assert np.array_equal(w.x_axis, c["dist"][sx:ex]) and np.array_equal(w.t_axis, c["t_axis"][st:et])
        assert w.veh_state is c["veh_states"][k] or np.array_equal(w.veh_state, c["veh_states"][k], equal_nan=True)
    assert np.array_equal(np.array([to_host(w.data).sum() for w in sel.windows]), g[case + "_sums"])
    if len(sel):
        assert np.array_equal(np.concatenate([w.veh_state_x for w in sel.windows]), g[case + "_vx"])
        assert np.array_equal(np.concatenate([w.veh_state_t for w in sel.windows]), g[case + "_vt"])


@pytest.mark.parametrize("case", CASES)
def test_selector_host_record(device, case):
    g = gio.load("select")
    c = gio.select_cases()[case]
    sel = _select(c, c["rec"])
    assert all(isinstance(w.data, np.ndarray) and w.data.dtype == np.float64 for w in sel.windows)
    _check(sel, c, g, case, lambda d: d)


@pytest.mark.parametrize("case", CASES)
def test_selector_device_record(device, case):
    import torch
    g = gio.load("select")
    c = gio.select_cases()[case]
    rec = torch.as_tensor(c["rec"], dtype=torch.float32, device=device)  # values exact in float32
    sel = _select(c, rec)
    assert all(w.data.is_cuda and w.data.dtype == torch.float32 for w in sel.windows)
    _check(sel, c, g, case, lambda d: d.double().cpu().numpy())
    if case != "odd":  # all windows one shape -> one contiguous device batch
        assert sel.batch is not None and sel.batch.shape[0] == len(sel)


def test_cut_windows_rejects_out_of_record(device):
    import torch

    from das_diff_veh_amd import _lib
    rec = torch.zeros((8, 100), dtype=torch.float32, device=device)
    out = torch.full((1, 4, 30), 7.0, dtype=torch.float32, device=device)
    starts = torch.tensor([80], dtype=torch.int64, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    _lib.call("dvh_cut_windows", _lib.ptr(rec), 0, 8, 100, 100, _lib.ptr(starts), 1, 2, 4, 30, _lib.ptr(out), 0,
              _lib.ptr(status), _lib.stream_of(device))
    assert int(status.item()) == 1 and bool((out == 7.0).all())
    with pytest.raises(_lib.DvhError):
        _lib.call("dvh_cut_windows", _lib.ptr(rec), 0, 8, 100, 100, _lib.ptr(starts), 1, 6, 4, 30, _lib.ptr(out), 0,
                  _lib.ptr(status), _lib.stream_of(device))
