"""GPU parity of the continuous-record preprocessing:
TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71) against the
reference's outputs (tests/golden/prep.npz): bandpass, the empty / noisy trace imputation quirks
(argmax -> trace 0 when nothing qualifies; a neighbour SUM) and the per-trace L2 norm."""
import numpy as np
import pytest

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
CASES = ["plain", "dead", "spike", "dead_last", "dead_first_spike"]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("method", ["surface_wave", "xcorr"])
def test_surface_wave_preprocessing(device, case, method):
    from das_diff_veh_amd.preprocess import surface_wave_preprocessing
    g = gio.load("prep")
    x = g[case + "_in"].astype(np.float64)
    got, idx = surface_wave_preprocessing(x, float(g["dt"]), method=method, return_indices=True)
    ref = g[f"{case}_{method}"]
    assert got.dtype == np.float64 and got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-10 * np.abs(ref).max(), case
    assert idx[0] == int(g[case + "_idx"][0])
    assert np.array_equal(x, g[case + "_in"].astype(np.float64))  # input untouched (data.copy())


def test_preprocessing_device_tensor_float32(device):
    import torch

    from das_diff_veh_amd.preprocess import surface_wave_preprocessing
    g = gio.load("prep")
    t = torch.as_tensor(g["dead_in"], device=device)  # float32 stays float32 on the device
    got = surface_wave_preprocessing(t, float(g["dt"]))
    assert got.is_cuda and got.dtype == torch.float32
    ref = g["dead_surface_wave"]
    assert np.abs(got.double().cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("case", CASES)
def test_float32_record_keeps_its_dtype(device, case):
    """A float32 host record: the reference's data.copy() stays float32 (filter output stored in float32,
    imputation and norm in float32); so does ours, against the reference's float32 run (prep.npz)."""
    from das_diff_veh_amd.preprocess import surface_wave_preprocessing
    g = gio.load("prep")
    x = g[case + "_in"]
    assert x.dtype == np.float32
    got = surface_wave_preprocessing(x, float(g["dt"]))
    ref = g[case + "_surface_wave_f32"]
    assert got.dtype == np.float32 and got.shape == ref.shape
    assert np.abs(got.astype(np.float64) - ref).max() <= 2e-6 * np.abs(ref).max(), case
