"""The ctypes stubs printed in INTEGRATION.md §2b (VirtualShotGather's body) and §2b' (bandpass_data) are runnable
and give the reference's outputs."""
import os
import re

import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source(section="### 2b."):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split(section, 1)[1]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_integration_stub_matches_golden(device, monkeypatch):
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md#2b", "exec"), ns)
    g = gio.load("vsg_w500")
    win = SurfaceWaveWindow(**gio.pass_arrays(g, 0))
    xcf, gx, gt = ns["construct_both_sides_gpu"](win, include_other_side=True, pivot=700, start_x=500, end_x=900,
                                                 wlen=2)
    assert gio.gather_rel_err(xcf, g["xcf_norm_2s"][0]) < 1e-4


def test_bandpass_stub_matches_reference(device, monkeypatch):
    """§2b' on the prep fixture's record (tests/golden/prep.npz) in float64 and float32, against bandpass_data's
    scipy.signal.sosfiltfilt (modules/utils.py:179-189): the matrix-pipe form for 1.2-30 Hz (pole radius 0.9956)
    and the recursion for 0.08-1 Hz (past the pole-radius gate)."""
    import numpy as np
    import torch

    from oracle import preprocess as oprep
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(_stub_source("### 2b'."), "INTEGRATION.md#2b'", "exec"), ns)
    g = gio.load("prep")
    dt = float(g["dt"])
    for dtype, tol in ((np.float64, 1e-10), (np.float32, 2e-6)):
        for flo, fhi in ((1.2, 30), (0.08, 1)):
            host = g["plain_in"].astype(dtype)
            got = ns["bandpass_data_gpu"](torch.as_tensor(host.copy(), device=device), dt, flo, fhi)
            ref = oprep.bandpass_data_scipy(host.astype(np.float64), dt, flo, fhi)
            assert got.dtype == torch.from_numpy(host).dtype
            assert np.abs(got.double().cpu().numpy() - ref).max() <= tol * np.abs(ref).max(), (dtype, flo, fhi)
