"""The host -> device window staging of the drop-in classes (device.stage_windows): pinned double buffers,
thread-parallel host copies, asynchronous H2D on a side stream, float64 -> float32 on the device.  The
staged batch equals the plain np.stack(...).astype(float32) copy bit for bit, over many chunks."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_stage_windows_matches_plain_copy(device, dtype, monkeypatch):
    import torch

    from das_diff_veh_amd import device as dv
    rng = np.random.default_rng(3)
    hosts = [rng.standard_normal((60, 550)).astype(dtype) for _ in range(23)]
    hosts[4][3, 7] = np.nan
    hosts[9][0, 0] = np.inf
    hosts[10][:] = 1e-42 if dtype == np.float32 else 1e-300  # subnormal / underflow to 0 in float32
    monkeypatch.setattr(dv, "STAGE_BYTES", 5 * hosts[0].nbytes)  # 5 windows per chunk: 5 chunks, both buffers reused
    got = dv.to_device_f32(hosts, device)
    ref = np.stack([h.astype(np.float32) for h in hosts])
    g = got.cpu().numpy()
    assert g.dtype == np.float32 and g.shape == ref.shape
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))
    # the caller's arrays may change right after the call returns
    hosts[0][:] = 0
    torch.cuda.synchronize()
    assert np.array_equal(got[0].cpu().numpy(), ref[0])
