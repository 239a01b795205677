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


def test_fk_grid_small_batch_split_k(device):
    """A few gathers (the bench's class stacks: 5 blocks of tdft_rows_kernel's 4-wave form) take its K-split form
    (4 wave groups, group sums added in order): |FK| equals the same gathers' |FK| inside a large batch (the
    single-group form) to 1e-12 of the grid's peak, and a float64 NumPy fk of the reference's expression
    (modules/utils.py:236-248) to 1e-11."""
    import torch

    from das_diff_veh_amd.disp import DispPlan, fk_grid
    rng = np.random.default_rng(31)
    nch, nt, dx, dt = 25, 1000, 8.16, 0.004
    plan = DispPlan(nch, nt, dx, dt, np.linspace(2.0, 25.0, 242), np.linspace(200.0, 1200.0, 1000))
    big = rng.standard_normal((300, nch, nt)).astype(np.float32)
    small = torch.as_tensor(big[:2], device=device)
    fk_small = fk_grid(small, plan).cpu().numpy()
    fk_big = fk_grid(torch.as_tensor(big, device=device), plan)[:2].cpu().numpy()
    peak = np.abs(fk_big).max()
    assert np.abs(fk_small - fk_big).max() <= 1e-12 * peak
    nf, nk = 2 ** (1 + int(np.ceil(np.log2(nt)))), 2 ** (1 + int(np.ceil(np.log2(nch))))
    assert (nf, nk) == (plan.nf, plan.nk)
    for b in range(2):
        full = np.abs(np.fft.fftshift(np.fft.fft2(big[b].astype(np.float64), s=[nk, nf])))
        ref = full[plan.m_lo:plan.m_lo + plan.n_kb, plan.j_lo:plan.j_lo + plan.n_fb]
        assert np.abs(fk_small[b] - ref).max() <= 1e-11 * np.abs(ref).max()
