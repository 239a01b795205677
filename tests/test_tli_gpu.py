"""GPU parity of the imaging half of TimeLapseImaging end to end (apis/timeLapseImaging.py:50-71,
166-201; SURVEY §8(f) rows 2-3, flavour B): a continuous record is preprocessed on the device, one
window per isolated pass is cut on the device, every window is muted along its trajectory and imaged
(naive dispersion) in one batch, and the mean f-v image is compared with the reference's
(tests/golden/tli.npz, same f-v contract as test_disp_gpu: rel-err 1e-4, picks on the maximum)."""
import numpy as np
import pytest

from tests import golden_io as gio
from tests.test_disp_gpu import _check

pytestmark = pytest.mark.gpu


def _tli(device_record=False):
    import torch

    from das_diff_veh_amd.apis.timeLapseImaging import TimeLapseImaging
    c = gio.select_cases()["short"]
    g = gio.load("tli")
    data = c["rec"].copy()
    if device_record:
        data = torch.as_tensor(data, device="cuda")
    obj = TimeLapseImaging(data, g["x_axis"], c["t_axis"])
    obj.set_tracking(c["veh_states"], c["start_x_tracking"], c["dist_trk"], c["t_trk"])
    obj.select_surface_wave_windows(c["x0"], **c["kw"])
    obj.get_images(mute_offset=300, start_x=560, end_x=680)
    return obj, g, c


def test_time_lapse_imaging_flavour_b(device):
    obj, g, c = _tli()
    assert len(obj.sw_selector) == int(g["n_windows"])
    _check(obj.images.images[0].disp.fv_map, g["fv_first"])
    _check(obj.images.avg_image.disp.fv_map, g["fv_avg"])
    assert np.array_equal(obj.qs_selector.windows[0].data, g["qs_first"])  # raw-data windows: exact copies
    assert not any(w.muted_along_traj for w in obj.sw_selector.windows)  # muted on a copy, like the reference


def test_time_lapse_imaging_device_record(device):
    obj, g, _ = _tli(device_record=True)
    assert obj.data_for_imaging.is_cuda and obj.sw_selector.batch is not None
    _check(obj.images.avg_image.disp.fv_map, g["fv_avg"])


def test_track_cars_is_outside_the_hot_path():
    from das_diff_veh_amd.apis.timeLapseImaging import TimeLapseImaging
    obj = TimeLapseImaging.__new__(TimeLapseImaging)
    with pytest.raises(NotImplementedError):
        obj.track_cars(0, 1, {})
