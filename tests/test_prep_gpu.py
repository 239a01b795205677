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


@pytest.mark.parametrize("form", ["recursion", "matrix"])
@pytest.mark.parametrize("n_rows,n_t,dtype,pad", [(640, 28000, np.float64, 0), (256, 140000, np.float32, 24)])
def test_sosfiltfilt_long_blocks_and_strided_rows(device, n_rows, n_t, dtype, pad, form):
    """Both forms through the C ABI: dvh_sosfiltfilt (the block recursion, blocks longer than 32 samples: the block
    length grows with the record, L = 96 and 160 here, with the longer A^L transition) and dvh_sosfiltfilt_planned
    (the matrix-pipe form: 64-sample blocks, a record past the LDS-resident scan's 240 blocks, so its staged scan);
    the float32 case on rows of a wider buffer (row stride n_t + 2 pad, the columns outside the rows untouched).
    Against scipy.signal.sosfiltfilt as bandpass_data calls it (oracle/preprocess.py): 1e-10 in float64, 2e-6 in
    float32."""
    import torch

    from das_diff_veh_amd import _lib
    from das_diff_veh_amd.preprocess import _design
    from oracle import preprocess as oprep
    dt = 0.004
    rng = np.random.default_rng(n_t)
    t = np.arange(n_t) * dt
    host = (rng.standard_normal((n_rows, n_t)) * 0.1 + np.sin(2 * np.pi * 7.0 * t)[None, :]).astype(dtype)
    buf = np.full((n_rows, n_t + 2 * pad), 3.5, dtype)
    buf[:, pad:pad + n_t] = host
    dev = torch.from_numpy(buf).to(device)
    rows = dev[:, pad:pad + n_t]
    sos, padlen, sos_t, zi_t = _design(dt, 1.2, 30, device)
    nbytes = int(_lib.load().dvh_sosfiltfilt_workspace(n_rows, n_t, len(sos), padlen))
    work = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)
    if form == "recursion":
        _lib.call("dvh_sosfiltfilt", _lib.ptr(rows), 0 if dtype == np.float32 else 1, n_rows, rows.stride(0), n_t,
                  _lib.ptr(sos_t), len(sos), padlen, _lib.ptr(zi_t), _lib.ptr(work), _lib.stream_of(device))
    else:
        plan = torch.empty(int(_lib.load().dvh_sosfiltfilt_plan_bytes(len(sos))) // 8, dtype=torch.float64,
                           device=device)
        _lib.call("dvh_sosfiltfilt_plan", _lib.ptr(sos_t), len(sos), _lib.ptr(zi_t), n_t, padlen, _lib.ptr(plan),
                  _lib.stream_of(device))
        _lib.call("dvh_sosfiltfilt_planned", _lib.ptr(rows), 0 if dtype == np.float32 else 1, n_rows, rows.stride(0),
                  n_t, _lib.ptr(sos_t), len(sos), padlen, _lib.ptr(zi_t), _lib.ptr(plan), _lib.ptr(work),
                  _lib.stream_of(device))
    got = dev.cpu().numpy()
    ref = oprep.bandpass_data_scipy(host.astype(np.float64), dt, 1.2, 30)
    tol = 1e-10 if dtype == np.float64 else 2e-6
    assert np.abs(got[:, pad:pad + n_t].astype(np.float64) - ref).max() <= tol * np.abs(ref).max()
    if pad:
        assert np.all(got[:, :pad] == 3.5) and np.all(got[:, pad + n_t:] == 3.5)


def test_matrix_form_only_for_poles_clear_of_the_unit_circle(device):
    """The drop-in plans the matrix-pipe form for the 1.2-30 Hz design (pole radius 0.9956) and takes the recursion
    for 0.08-1 Hz (0.99973), whose block GEMMs would round to 5e-10 of the output (tests/test_disp_gpu.py's
    bandpass cases hold both to 1e-10)."""
    from das_diff_veh_amd import _lib
    from das_diff_veh_amd import preprocess as pp
    for (flo, fhi), planned in (((1.2, 30), True), ((0.08, 1), False)):
        sos, padlen, sos_t, zi_t = pp._design(0.004, flo, fhi, device)
        r = _lib.load().dvh_sos_pole_radius(np.ascontiguousarray(sos).ctypes.data, len(sos))
        assert (r <= pp.SOS_MFMA_MAX_POLE) == planned, (flo, fhi, r)
        plan = pp._plan((0.004, flo, fhi, str(device)), 3000, sos, padlen, sos_t, zi_t, device)
        assert (plan is not None) == planned


@pytest.mark.parametrize("n_rows,n_t", [(48, 130), (48, 700), (48, 4000), (48, 15500), (48, 16600), (45, 130),
                                          (47, 700)])
def test_matrix_form_record_lengths(device, n_rows, n_t):
    """The matrix-pipe form across the scans it dispatches to: records of 4 blocks (one group holds every block),
    mid-size records (groups of 1-3 blocks, some of the 16 groups empty), 15 500 samples (16 groups of 16 blocks, the
    last partial: the matrix-pipe scan's limit) and 16 600 (past it: the staged scan); 45 x 130 and 47 x 700 leave a
    partial last tile of 16 columns spanning 3+ rows, whose padding columns (rows >= n_rows) must read nothing.
    float64 rows against scipy.signal.sosfiltfilt as bandpass_data calls it (1e-10)."""
    import torch

    from das_diff_veh_amd.preprocess import bandpass_inplace
    from oracle import preprocess as oprep
    rng = np.random.default_rng(n_t)
    dt = 0.004
    host = rng.standard_normal((n_rows, n_t)) + np.sin(2 * np.pi * 7.0 * np.arange(n_t) * dt)[None, :]
    dev = torch.from_numpy(host.copy()).to(device)
    bandpass_inplace(dev, dt, 1.2, 30)
    ref = oprep.bandpass_data_scipy(host, dt, 1.2, 30)
    assert np.abs(dev.cpu().numpy() - ref).max() <= 1e-10 * np.abs(ref).max()


def _planned_run(device, sos, host, plan_n_t):
    """dvh_sosfiltfilt_plan for a record of plan_n_t samples, then dvh_sosfiltfilt_planned on host's rows."""
    import scipy.signal
    import torch

    from das_diff_veh_amd import _lib
    from das_diff_veh_amd.preprocess import _padlen
    n_rows, n_t = host.shape
    padlen = _padlen(sos)
    sos_t = torch.from_numpy(np.ascontiguousarray(sos, dtype=np.float64)).to(device)
    zi_t = torch.from_numpy(np.ascontiguousarray(scipy.signal.sosfilt_zi(sos), dtype=np.float64)).to(device)
    dev = torch.from_numpy(host.copy()).to(device)
    nbytes = int(_lib.load().dvh_sosfiltfilt_workspace(n_rows, n_t, len(sos), padlen))
    work = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)
    plan = torch.empty(int(_lib.load().dvh_sosfiltfilt_plan_bytes(len(sos))) // 8, dtype=torch.float64, device=device)
    _lib.call("dvh_sosfiltfilt_plan", _lib.ptr(sos_t), len(sos), _lib.ptr(zi_t), plan_n_t, padlen, _lib.ptr(plan),
              _lib.stream_of(device))
    _lib.call("dvh_sosfiltfilt_planned", _lib.ptr(dev), 1, n_rows, dev.stride(0), n_t, _lib.ptr(sos_t), len(sos),
              padlen, _lib.ptr(zi_t), _lib.ptr(plan), _lib.ptr(work), _lib.stream_of(device))
    return dev.cpu().numpy()


def test_matrix_form_low_order_lds_resident_scan(device):
    """A 4-section design (butter(4, band)) on a 20 000-sample record: 314 blocks, past the matrix-pipe scan's 258 and
    inside the LDS-resident VALU scan's range at 8 state components (sosm_scanr_kernel, which the drop-in's 10-section
    design never reaches), against scipy.signal.sosfiltfilt at 1e-10."""
    import scipy.signal
    dt = 0.004
    sos = scipy.signal.butter(4, [1.2 * 2 * dt, 30 * 2 * dt], "bandpass", output="sos")
    assert len(sos) == 4
    rng = np.random.default_rng(4)
    n_t = 20000
    host = rng.standard_normal((40, n_t)) + np.sin(2 * np.pi * 7.0 * np.arange(n_t) * dt)[None, :]
    got = _planned_run(device, sos, host, n_t)
    ref = scipy.signal.sosfiltfilt(sos, host, axis=1)
    assert np.abs(got - ref).max() <= 1e-10 * np.abs(ref).max()


def test_plan_for_another_record_length_poisons_the_output(device):
    """A plan carries the group size its group transitions were formed for: planned for 4 000 samples and run on
    15 000 (another group size, carried groups in use), the output holds NaN instead of a silently wrong filter."""
    from das_diff_veh_amd.preprocess import butter_bandpass_sos
    sos = butter_bandpass_sos(0.004, 1.2, 30)
    host = np.random.default_rng(5).standard_normal((8, 15000))
    got = _planned_run(device, sos, host, 4000)
    assert np.isnan(got).any()
    ok = _planned_run(device, sos, host, 15000)
    assert np.isfinite(ok).all()
