"""GPU parity of the public fk (modules/utils.py:236-248): |fftshift(fft2(data, s=[nk, nf]))| and its
(fft_f, fft_k) axes against the reference's own output (tests/golden/fk.npz, make_golden.gen_fk)."""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["stack", "odd", "pow2"])
def test_fk_matches_reference(device, case):
    from das_diff_veh_amd.modules.utils import fk
    g = gio.load("fk")
    res, ff, kk = fk(g[case + "_data"], float(g[case + "_dx"]), float(g[case + "_dt"]))
    ref = g[case + "_fk"].astype(np.float64)
    assert res.shape == ref.shape
    # fp32 input, fp64 MFMA transform: rel <= 1e-4 of the grid's peak (north_star's gather tolerance)
    assert np.abs(res - ref).max() <= 1e-4 * np.abs(ref).max()
    assert np.array_equal(ff, g[case + "_f"]) and np.array_equal(kk, g[case + "_k"])
