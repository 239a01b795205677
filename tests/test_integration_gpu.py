"""The ctypes stub printed in INTEGRATION.md §2b is runnable and gives the reference's gathers."""
import os
import re

import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split("### 2b.", 1)[1]
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
