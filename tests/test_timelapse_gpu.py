"""Full-size parity of the time-lapse dispersion path (BASELINE configs[4], `bench.py --workload timelapse`):
512 gathers of 25 ch x 500 lags imaged on 512 velocities x 1,000 frequencies in ONE batch.

* The product dispatch (time DFT on `tdft_rows_kernel`, f-v on `fv_mfma_kernel`) against the cell-staged
  VALU f-v kernel on the same |FK| grids, over all 512 images: both form the same float32 bilinear
  samples (modules/utils.py:466-472), so the images may differ only by the Savitzky-Golay summation order
  (float64): rel <= 1e-6 per image, and every MFMA pick is a maximum of the VALU image up to that bound.
* Six of the images against the oracle's map_fv (modules/utils.py:457-475): rel <= 1e-4, picks per the
  SURVEY §8(d) tie rule.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
B, NV, NF = 512, 512, 1000
DX, DT = 8.16, 0.003999999999997783


@pytest.fixture(scope="module")
def job(device):
    import torch

    from das_diff_veh_amd.disp import DispPlan, _use_mfma, fk_grid
    from das_diff_veh_amd.synth import synth_gathers
    freqs, vels = np.linspace(1.0, 25.0, NF), np.linspace(200.0, 1200.0, NV)
    plan = DispPlan(25, 500, DX, DT, freqs, vels)
    assert _use_mfma(plan, B)
    data = synth_gathers(B, 25, 500, DX, DT, device, seed=7)
    FK = fk_grid(data, plan)
    torch.cuda.synchronize()
    return dict(plan=plan, data=data, FK=FK, freqs=freqs, vels=vels)


def test_mfma_fv_matches_valu_fv_on_the_full_batch(job, monkeypatch):
    import torch

    from das_diff_veh_amd.disp import fv_from_fk
    plan, FK = job["plan"], job["FK"]
    got = fv_from_fk(FK, plan)  # product dispatch: fv_mfma_kernel
    monkeypatch.setenv("DVH_FV_MFMA", "0")
    monkeypatch.setenv("DVH_FV_CELLS", "1")
    ref = fv_from_fk(FK, plan)  # cell-staged fv_tile_kernel
    torch.cuda.synchronize()
    peak = ref.abs().amax(dim=(1, 2))
    rel = (got - ref).abs().amax(dim=(1, 2)) / peak
    assert float(rel.max()) <= 1e-6, float(rel.max())
    picks = got.argmax(dim=1)                                   # [B, NF]
    at_pick = torch.gather(ref, 1, picks[:, None, :])[:, 0, :]  # the VALU image at the MFMA pick
    colmax = ref.amax(dim=1)
    assert bool(((colmax - at_pick) <= 1e-6 * peak[:, None]).all())
    exact = float((at_pick == colmax).float().mean())
    assert exact > 0.999, exact
    print(f"max rel diff {float(rel.max()):.2e}, picks exactly a column max: {exact:.6f}")


def test_mfma_fv_matches_oracle_on_sampled_images(job):
    from das_diff_veh_amd.disp import fv_from_fk
    from oracle import disp as odisp
    got = fv_from_fk(job["FK"], job["plan"])
    host = job["data"].double().cpu().numpy()
    for b in (0, 1, 137, 256, 400, B - 1):
        ref = odisp.map_fv(host[b], DX, DT, job["freqs"], job["vels"])
        g = got[b].double().cpu().numpy()
        assert np.abs(g - ref).max() / np.abs(ref).max() < 1e-4, b
        assert np.all(odisp.pick_ok(ref, g.argmax(axis=0))), b
