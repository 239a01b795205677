"""GPU parity of the batched f-v sampling kernel (fv_batch_kernel) on BASELINE configs[4]'s grid:
512 velocities x 1,000 frequencies, many images per launch (weights reused across the images of a
block), against the oracle's map_fv (modules/utils.py:457-475): rel-err <= 1e-4, picks per the
SURVEY §8(d) tie rule."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.mark.parametrize("mode", [None, ("DVH_FV_TILE", "2"), ("DVH_FV_TILE", "0"), ("DVH_FV_G", "3"),
                                  ("DVH_FV_G", "16"), ("DVH_FV_TG", "3"), ("DVH_FV_G", "0"), ("DVH_FV_CELLS", "1"),
                                  ("DVH_FV_CELLS", "0"), ("DVH_FV_MFMA", "1"), ("DVH_FV_MG", "3")])
@pytest.mark.parametrize("B,nv,nf", [(40, 512, 1000), (7, 300, 242), (5, 64, 1001), (3, 61, 25), (4, 33, 413),
                                     (3, 17, 32), (2, 16, 40), (5, 70, 47)])
def test_fv_batch_vs_oracle(device, monkeypatch, B, nv, nf, mode):
    """mode: kernel selection read at each launch -- None = default dispatch, DVH_FV_TILE=2 -> always
    the frequency-tiled kernel, DVH_FV_TILE=0 -> batched / per-image dispatch, DVH_FV_G = images per block of the batched kernel (0: per-image
    kernel), DVH_FV_TG = images per block of the tiled kernel, DVH_FV_MFMA=1 -> the MFMA-filter kernel where
    it applies (nF >= 32), DVH_FV_MG = its images per block."""
    if mode is not None:
        if mode[0] == "DVH_FV_G":
            monkeypatch.setenv("DVH_FV_TILE", "0")
        if mode[0] == "DVH_FV_TG":
            monkeypatch.setenv("DVH_FV_TILE", "2")
        if mode == ("DVH_FV_CELLS", "1"):  # also split the images over several blocks
            monkeypatch.setenv("DVH_FV_TG", "3")
        if mode[0] == "DVH_FV_MG":  # MFMA-filter kernel, 3 images per block
            monkeypatch.setenv("DVH_FV_MFMA", "1")
        monkeypatch.setenv(*mode)
    from das_diff_veh_amd.disp import DispPlan, fv_maps
    from das_diff_veh_amd.synth import synth_gathers
    from oracle import disp as odisp
    nch, nt, dx, dt = 25, 500, 8.16, 0.003999999999997783
    freqs, vels = np.linspace(1.0, 25.0, nf), np.linspace(200.0, 1200.0, nv)
    data = synth_gathers(B, nch, nt, dx, dt, device, seed=B)
    got = fv_maps(data, DispPlan(nch, nt, dx, dt, freqs, vels)).double().cpu().numpy()
    host = data.double().cpu().numpy()
    for b in sorted({0, 1, B // 2, B - 1}):
        ref = odisp.map_fv(host[b], dx, dt, freqs, vels)
        assert np.abs(got[b] - ref).max() / np.abs(ref).max() < TOL, b
        assert np.all(odisp.pick_ok(ref, got[b].argmax(axis=0))), b
