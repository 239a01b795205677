"""Generate the golden vectors under tests/golden/ by running the REFERENCE in this container.

Run once, here (the survey container), never on the GPU box:

    python tests/golden/make_golden.py

It imports NohPei/das_diff_veh from /root/reference with the shims SURVEY.md §8(c) lists
(stub modules for obspy/segyio/cv2, which the hot path never calls; numpy aliases for the
``from scipy import arange, array, exp`` line removed from SciPy; an ``interp2d`` replacement,
since SciPy >= 1.14 raises ``NotImplementedError`` for it and names ``RectBivariateSpline`` on a
regular grid as the bug-for-bug replacement).  Nothing is written into /root/reference.

Only data leaves this script: int16-quantised inputs (exact in fp32) and the reference's outputs.
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np
import scipy
import scipy.interpolate
import scipy.signal

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from das_diff_veh_amd.synth import synth_pass, DT_W500, DT_W499  # noqa: E402
from tests.golden_io import select_cases  # noqa: E402

REF = "/root/reference"


class _Interp2dShim:
    """interp2d(x, y, z, kind='linear') on a rectangular grid, as SciPy < 1.14 evaluated it.

    regrid_smth with kx = ky = 1 and s = 0 reproduces the data at the knots; bisplev clamps
    queries to the grid and __call__ sorts the query vectors (mergesort) before evaluating.
    """

    def __init__(self, x, y, z, kind="linear"):
        assert kind == "linear"
        x = np.ravel(x)
        y = np.ravel(y)
        z = np.asarray(z)
        assert z.shape == (len(y), len(x))
        self.spl = scipy.interpolate.RectBivariateSpline(x, y, z.T, kx=1, ky=1, s=0)

    def __call__(self, x, y):
        x = np.sort(np.atleast_1d(x), kind="mergesort")
        y = np.sort(np.atleast_1d(y), kind="mergesort")
        z = np.atleast_2d(self.spl(x, y)).T
        if len(z) == 1:
            z = z[0]
        return np.array(z)


def import_reference():
    import matplotlib
    matplotlib.use("Agg")
    for name in ("obspy", "obspy.signal", "obspy.signal.filter", "segyio", "cv2"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["obspy.signal.filter"].bandpass = None
    scipy.arange, scipy.array, scipy.exp = np.arange, np.array, np.exp
    scipy.interpolate.interp2d = _Interp2dShim
    sys.path.insert(0, REF)
    import apis.data_classes as dc
    import apis.virtual_shot_gather as vsg
    import apis.dispersion_classes as dcl
    import apis.imaging_classes as ic
    import modules.utils as ut
    return types.SimpleNamespace(dc=dc, vsg=vsg, dcl=dcl, ic=ic, ut=ut)


def ref_window(ref, p, dtype=np.float64):
    return ref.dc.SurfaceWaveWindow(
        data=p["data"].astype(dtype), x_axis=p["x_axis"], t_axis=p["t_axis"], veh_state=p["veh_state"],
        start_x_tracking=p["start_x_tracking"],
        distance_along_fiber_tracking=p["distance_along_fiber_tracking"],
        t_axis_tracking=p["t_axis_tracking"])


def pack_inputs(passes, prefix=""):
    out = {}
    out[prefix + "q"] = np.stack([p["q"] for p in passes])
    out[prefix + "x_axis"] = np.stack([p["x_axis"] for p in passes])
    out[prefix + "t_axis"] = np.stack([p["t_axis"] for p in passes])
    out[prefix + "veh_state"] = np.stack([p["veh_state"] for p in passes])
    out[prefix + "start_x_tracking"] = np.array([p["start_x_tracking"] for p in passes])
    out[prefix + "distance_along_fiber_tracking"] = passes[0]["distance_along_fiber_tracking"]
    out[prefix + "t_axis_tracking"] = np.stack([p["t_axis_tracking"] for p in passes])
    return out


def gen_vsg(ref):
    """Per-pass gathers, the class stack and its dispersion image (call stack A)."""
    kw = dict(pivot=700, start_x=500, end_x=900, wlen=2)
    passes = [synth_pass(100 + i) for i in range(5)]
    wins = [ref_window(ref, p) for p in passes]
    out = pack_inputs(passes)

    # ImagesFromWindows.get_images path: norm=False, include_other_side=True (imaging_classes.py:137)
    images = ref.ic.VirtualShotGathersFromWindows(wins)
    images.get_images(include_other_side=True, **kw)
    out["xcf"] = np.stack([im.XCF_out for im in images.images])
    out["gather_x_axis"] = images.images[0].x_axis
    out["gather_t_axis"] = images.images[0].t_axis
    out["stack"] = images.avg_image.XCF_out
    images.avg_image.compute_disp_image(end_x=0, start_x=-200)
    out["fv_map"] = images.avg_image.disp.fv_map
    out["fv_freqs"] = images.avg_image.disp.freqs
    out["fv_vels"] = images.avg_image.disp.vels

    # VirtualShotGather called directly: norm=True default; one-sided and two-sided
    out["xcf_norm_2s"] = np.stack([ref.vsg.VirtualShotGather(w, include_other_side=True, **kw).XCF_out
                                   for w in wins[:1]])
    out["xcf_norm_1s"] = np.stack([ref.vsg.VirtualShotGather(w, include_other_side=False, **kw).XCF_out
                                   for w in wins[:1]])
    out["xcf_nonorm_1s"] = np.stack([ref.vsg.VirtualShotGather(w, include_other_side=False, norm=False, **kw).XCF_out
                                     for w in wins[:1]])
    # raw correlation scale: norm=False, norm_amp=False keeps the data / ||data||_F factor
    out["xcf_raw_2s"] = np.stack([ref.vsg.VirtualShotGather(w, include_other_side=True, norm=False,
                                                            norm_amp=False, **kw).XCF_out for w in wins[:1]])
    # dispersion of the stack with the per-trace L1 normalisation (map_fv norm=True)
    im = images.avg_image
    s = np.abs(im.x_axis - (-200)).argmin()
    e = np.abs(im.x_axis - 0).argmin()
    d = ref.ut.Dispersion(im.XCF_out[s:e + 1], 8.16, im.t_axis[1] - im.t_axis[0],
                          freqs=np.arange(0.8, 25, 0.1), vels=np.arange(200, 1200), norm=True)
    out["fv_map_l1"] = d.fv_map
    return out


def gen_vsg_w499(ref):
    """dt slightly above 0.004: w = 499 (prime), nsamp = 999, hop = 249."""
    kw = dict(pivot=700, start_x=500, end_x=900, wlen=2)
    passes = [synth_pass(200 + i, t0=DT_W499) for i in range(2)]
    wins = [ref_window(ref, p) for p in passes]
    out = pack_inputs(passes)
    images = ref.ic.VirtualShotGathersFromWindows(wins)
    images.get_images(include_other_side=True, **kw)
    out["xcf"] = np.stack([im.XCF_out for im in images.images])
    out["stack"] = images.avg_image.XCF_out
    out["gather_t_axis"] = images.images[0].t_axis
    images.avg_image.compute_disp_image(end_x=0, start_x=-200)
    out["fv_map"] = images.avg_image.disp.fv_map
    return out


def gen_vsg_edge(ref):
    """Edge cases: empty/wrapped slices, truncated windows, pivot near the aperture edge."""
    out = {}
    cases = [
        # (name, synth kwargs, vsg kwargs)
        ("early", dict(seed=300, tc_offset=-7.2), dict(pivot=700, start_x=500, end_x=900)),   # other side empty -> NaN side
        ("late", dict(seed=301, tc_offset=5.5), dict(pivot=700, start_x=500, end_x=900)),     # fwd window truncated
        ("slow", dict(seed=302, speed=12.0), dict(pivot=700, start_x=500, end_x=900)),        # far rows leave the window
        ("p680", dict(seed=303, pivot=680.0), dict(pivot=680, start_x=480, end_x=880)),
        ("narrow", dict(seed=304), dict(pivot=700, start_x=690, end_x=760)),
        ("wlen1", dict(seed=305), dict(pivot=700, start_x=500, end_x=900, wlen=1, time_window_to_xcorr=3, delta_t=0.5)),
    ]
    for name, skw, vkw in cases:
        seed = skw.pop("seed")
        p = synth_pass(seed, **skw)
        w = ref_window(ref, p)
        for k, v in pack_inputs([p]).items():
            out[f"{name}_{k}"] = v
        g = ref.vsg.VirtualShotGather(w, include_other_side=True, norm=False, **vkw)
        out[f"{name}_xcf"] = g.XCF_out
        out[f"{name}_gx"] = g.x_axis
        out[f"{name}_gt"] = g.t_axis
        out[f"{name}_kw"] = np.array(repr(vkw))
    # dt == 0.004 exactly: int(2 // dt) = 499 != int(2 / dt) = 500 -> the reference raises ValueError
    p = synth_pass(306, t0=0.0)
    try:
        ref.vsg.VirtualShotGather(ref_window(ref, p), include_other_side=True, norm=False,
                                  pivot=700, start_x=500, end_x=900)
        out["dt004_raises"] = np.array(False)
    except ValueError:
        out["dt004_raises"] = np.array(True)
    return out


def gen_disp(ref):
    """Per-pass dispersion flavour (SurfaceWaveDispersion, dispersion_classes.py:9-65) and mutes."""
    out = {}
    passes = [synth_pass(400 + i, n_t=2048) for i in range(3)]
    for k, v in pack_inputs(passes).items():
        out[k] = v
    freqs = np.arange(0.8, 25, 0.1)
    vels = np.arange(200, 1200, 2)
    wins = [ref_window(ref, p) for p in passes]
    naive = [ref.dcl.SurfaceWaveDispersion(w, freqs=freqs, vels=vels, method="naive", norm=False,
                                           start_x=500, end_x=800) for w in wins]
    out["naive_fv"] = np.stack([d.disp.fv_map for d in naive])
    out["naive_stack"] = (sum(naive) / len(naive)).disp.fv_map
    out["naive_l1_fv"] = ref.dcl.SurfaceWaveDispersion(wins[0], freqs=freqs, vels=vels, method="naive", norm=True,
                                                       start_x=500, end_x=800).disp.fv_map
    out["smart_fv"] = ref.dcl.SurfaceWaveDispersion(wins[1], freqs=freqs, vels=vels, method="smart",
                                                    norm=False).disp.fv_map
    # DispersionImagesFromWindows.get_images: mute_along_traj(offset=300) on a copy, naive disp, mean
    imgs = ref.ic.DispersionImagesFromWindows(wins)
    imgs.get_images(mute_offset=300, freqs=freqs, vels=vels, method="naive", start_x=500, end_x=800)
    out["muted_stack"] = imgs.avg_image.disp.fv_map
    out["freqs"] = freqs
    out["vels"] = vels
    # mute outputs themselves
    import copy
    w = copy.deepcopy(wins[2])
    w.mute_along_traj(offset=300)
    out["mute_traj_300"] = w.data.astype(np.float32)
    w = copy.deepcopy(wins[2])
    w.mute_along_time(alpha=0.3)
    out["mute_time_03"] = w.data.astype(np.float32)
    return out


def gen_bandpass(ref):
    """bandpass_data (modules/utils.py:179-189) as called at apis/timeLapseImaging.py:60."""
    rng = np.random.default_rng(500)
    n_ch, n_t = 8, 3000
    t = np.arange(n_t) * 0.004
    x = np.zeros((n_ch, n_t))
    for f in (0.3, 0.9, 2.0, 7.5, 18.0, 33.0, 60.0):
        x += np.cos(2 * np.pi * f * t[None, :] + rng.uniform(0, 6.28, (n_ch, 1)))
    x += 0.3 * rng.standard_normal((n_ch, n_t))
    q = np.round(x / 2 ** -12).astype(np.int16)
    data = q.astype(np.float64) * 2 ** -12
    y = data.copy()
    ref.ut.bandpass_data(y, 0.004, 1.2, 30)
    y2 = data.copy()
    ref.ut.bandpass_data(y2, 0.004, 0.08, 1)
    return dict(q=q, dt=np.array(0.004), out_1p2_30=y, out_0p08_1=y2)


def gen_ridge(ref):
    """extract_ridge_ref_idx (modules/utils.py:621-678) on the vsg_w500 class image, and
    bootstrap_disp (apis/imaging_classes.py:8-48) with random.seed fixed, on the 5 fixture passes."""
    import random
    kw = dict(pivot=700, start_x=500, end_x=900, wlen=2)
    passes = [synth_pass(100 + i) for i in range(5)]
    wins = [ref_window(ref, p) for p in passes]
    images = ref.ic.VirtualShotGathersFromWindows(wins)
    images.get_images(include_other_side=True, **kw)
    images.avg_image.compute_disp_image(end_x=0, start_x=-200)
    d = images.avg_image.disp
    freqs, vels, fv = d.freqs, d.vels, d.fv_map
    out = dict(fv_map=fv, freqs=freqs, vels=vels)
    m0 = (freqs >= 2.5) & (freqs < 14)
    out["walk"] = ref.ut.extract_ridge_ref_idx(freqs[m0], vels, fv[:, m0], ref_freq_idx=80 - int(np.sum(freqs < 2.5)),
                                                sigma=25, vel_max=800)
    m1 = (freqs >= 10) & (freqs < 15)
    mode1 = scipy.interpolate.interp1d([10, 12, 13, 14, 15, 16], [530, 470, 450, 430, 410, 391])
    out["refvel"] = ref.ut.extract_ridge_ref_idx(freqs[m1], vels, fv[:, m1], ref_freq_idx=130 - int(np.sum(freqs < 10)),
                                                  sigma=50, vel_max=800, ref_vel=mode1)
    out["refvel_f"] = np.array([10, 12, 13, 14, 15, 16], float)
    out["refvel_v"] = np.array([530, 470, 450, 430, 410, 391], float)
    out["velmax"] = ref.ut.extract_ridge_ref_idx(freqs[m0], vels, fv[:, m0], sigma=25, vel_max=800)
    # a negative (Python) reference index: column nb - 7, then the reference's own loop order
    out["walk_neg7"] = ref.ut.extract_ridge_ref_idx(freqs[m0], vels, fv[:, m0], ref_freq_idx=-7, sigma=25, vel_max=800)
    # bootstrap: two modes (a walk and a reference-curve mode), bt_size 3 of the 4 drawable passes
    random.seed(11)
    rv, fq = ref.ic.bootstrap_disp(wins, 3, 4, [25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    out["boot_mode0"] = np.stack(rv[0])
    out["boot_mode1"] = np.stack(rv[1])
    out["boot_freqs"] = fq
    random.seed(11)
    out["boot_sel"] = np.array([random.sample(range(1, len(wins)), 3) for _ in range(4)])
    # the reference's f-v map of every resample (the same draws), for the per-pick parity of bootstrap_disp
    fvs = []
    for sel in out["boot_sel"]:
        imgs = ref.ic.VirtualShotGathersFromWindows([wins[i] for i in sel])
        imgs.get_images(pivot=700, start_x=500, end_x=900, wlen=2, include_other_side=True)
        imgs.avg_image.compute_disp_image(end_x=0, start_x=-150)
        fvs.append(imgs.avg_image.disp.fv_map)
    out["boot_fv"] = np.stack(fvs).astype(np.float32)
    return out


def gen_fk(ref):
    """fk (modules/utils.py:236-248): |fftshift(fft2(data, s=[nk, nf]))| and its axes, on the [-200, 0] m
    rows of the vsg_w500 class stack (the block compute_disp_image images) and on two quantised random
    blocks with non-power-of-two and power-of-two shapes."""
    kw = dict(pivot=700, start_x=500, end_x=900, wlen=2)
    wins = [ref_window(ref, synth_pass(100 + i)) for i in range(5)]
    images = ref.ic.VirtualShotGathersFromWindows(wins)
    images.get_images(include_other_side=True, **kw)
    im = images.avg_image
    s = np.abs(im.x_axis - (-200)).argmin()
    e = np.abs(im.x_axis - 0).argmin()
    out = {}
    rng = np.random.default_rng(700)
    cases = {"stack": (im.XCF_out[s:e + 1], 8.16, im.t_axis[1] - im.t_axis[0]),
             "odd": (np.round(rng.standard_normal((37, 777)) * 2 ** 10) / 2 ** 10, 4.08, 0.002),
             "pow2": (np.round(rng.standard_normal((32, 512)) * 2 ** 10) / 2 ** 10, 8.16, 0.004)}
    for name, (data, dx, dt) in cases.items():
        res, ff, kk = ref.ut.fk(data, dx, dt)
        out[name + "_data"] = np.asarray(data, dtype=np.float64)
        out[name + "_dx"], out[name + "_dt"] = np.array(dx), np.array(dt)
        out[name + "_fk"] = res.astype(np.float32)
        out[name + "_f"], out[name + "_k"] = ff, kk
    return out


def gen_prep(ref):
    """TimeLapseImaging._preprocessing_for_surface_waves (apis/timeLapseImaging.py:51-71) on a
    continuous record: bandpass, empty / noisy trace imputation (find_noise_idx, impute_noisy_trace,
    modules/utils.py:316-329), per-trace L2 norm.  Called unbound on a plain object holding the
    attributes it reads (the constructor's tracking preprocessing is outside the hot path)."""
    import apis.timeLapseImaging as tli
    rng = np.random.default_rng(600)
    n_ch, n_t, dt = 16, 2500, 0.004
    t = np.arange(n_t) * dt
    base = np.zeros((n_ch, n_t))
    for f in (0.5, 3.0, 8.0, 15.0, 40.0):
        base += 4.0 * np.cos(2 * np.pi * f * t[None, :] + rng.uniform(0, 6.28, (n_ch, 1)))
    base += 2.0 * rng.standard_normal((n_ch, n_t))
    cases = {
        "plain": lambda d: d,                                          # nothing qualifies: trace 0 <- trace 1
        "dead": lambda d: (d.__setitem__(7, 0.0), d)[1],               # empty trace 7 -> d[6] + d[8]
        "spike": lambda d: (d.__setitem__((13, slice(1000, 1010)), 400.0), d)[1],  # noisy trace 13
        "dead_last": lambda d: (d.__setitem__(n_ch - 1, 0.0), d)[1],   # empty last trace -> d[-2]
        "dead_first_spike": lambda d: (d.__setitem__(0, 0.0), d.__setitem__((5, 200), 900.0), d)[2],
    }
    out = dict(dt=np.array(dt))
    for name, mk in cases.items():
        d = mk(np.round(base * 2 ** 10) / 2 ** 10)
        out[name + "_in"] = d.astype(np.float32)  # multiples of 2**-10: exact in float32
        for method in ("surface_wave", "xcorr"):
            obj = types.SimpleNamespace(method=method, data=d.copy(), dt=dt, surface_wave_preprecessing_dict=None)
            tli.TimeLapseImaging._preprocessing_for_surface_waves(obj)
            out[f"{name}_{method}"] = obj.data_for_imaging
        bp = d.copy()
        ref.ut.bandpass_data(bp, dt, 1.2, 30)
        out[name + "_idx"] = np.array([ref.ut.find_noise_idx(bp, 5, empty_tr=True)])
        # a float32 record: data.copy() keeps float32, so the filter output is stored in float32 and the
        # imputation and the norm run in float32
        obj = types.SimpleNamespace(method="surface_wave", data=d.astype(np.float32), dt=dt,
                                    surface_wave_preprecessing_dict=None)
        tli.TimeLapseImaging._preprocessing_for_surface_waves(obj)
        assert obj.data_for_imaging.dtype == np.float32
        out[name + "_surface_wave_f32"] = obj.data_for_imaging
    return out


def gen_select(ref):
    """SurfaceWaveSelector (apis/data_classes.py:126-223): accepted vehicles, window index ranges and
    the cut data of every window (float64 record, deep-copied slices)."""
    out = {}
    for name, c in select_cases().items():
        sel = ref.dc.SurfaceWaveSelector(c["rec"], c["dist"], c["t_axis"], c["x0"], c["start_x_tracking"],
                                         c["veh_states"], c["dist_trk"], c["t_trk"], **c["kw"])
        rows = []
        for w in sel.windows:
            k = next(i for i in range(c["veh_states"].shape[0]) if w.veh_state is c["veh_states"][i]
                     or np.array_equal(w.veh_state, c["veh_states"][i], equal_nan=True))
            sx = int(np.flatnonzero(c["dist"] == w.x_axis[0])[0])
            st = int(np.flatnonzero(c["t_axis"] == w.t_axis[0])[0])
            rows.append([k, sx, sx + w.data.shape[0], st, st + w.data.shape[1]])
            assert np.array_equal(w.data, c["rec"][sx:sx + w.data.shape[0], st:st + w.data.shape[1]])
        out[name + "_windows"] = np.array(rows, dtype=np.int64).reshape(-1, 5)
        out[name + "_sums"] = np.array([w.data.sum() for w in sel.windows])
        out[name + "_vx"] = np.concatenate([w.veh_state_x for w in sel.windows]) if sel.windows else np.zeros(0)
        out[name + "_vt"] = np.concatenate([w.veh_state_t for w in sel.windows]) if sel.windows else np.zeros(0)
    return out


def gen_tli(ref):
    """TimeLapseImaging's imaging half end to end (apis/timeLapseImaging.py:50-71, 166-201), flavour B:
    preprocessing of the continuous record, SurfaceWaveSelector, DispersionImagesFromWindows (trajectory
    mute, naive dispersion per window, mean).  Called unbound on a plain object holding the tracking
    results (the tracker itself is outside the hot path)."""
    import apis.timeLapseImaging as tli
    c = select_cases()["short"]
    x_axis = 449.0 + np.arange(c["rec"].shape[0])
    obj = types.SimpleNamespace(method="surface_wave", data=c["rec"].copy(), dt=c["t_axis"][1] - c["t_axis"][0],
                                t_axis=c["t_axis"], x_axis=x_axis, distances_along_fiber=(x_axis - 400) * 8.16,
                                surface_wave_preprecessing_dict=None, start_x=c["start_x_tracking"],
                                veh_states=c["veh_states"], dist_along_fiber_tracking=c["dist_trk"],
                                t_axis_tracking=c["t_trk"])
    T = tli.TimeLapseImaging
    T._preprocessing_for_surface_waves(obj)
    T.select_surface_wave_windows(obj, c["x0"], **c["kw"])
    T.get_images(obj, mute_offset=300, start_x=560, end_x=680)
    return dict(x_axis=x_axis, n_windows=np.array(len(obj.sw_selector.windows)),
                fv_avg=obj.images.avg_image.disp.fv_map, fv_first=obj.images.images[0].disp.fv_map,
                qs_first=obj.qs_selector.windows[0].data)


def gen_workflow(ref):
    """The xcorr flavour of the daily workflow, ImagingWorkflowOneDirectory.imaging (apis/imaging_workflow.py:33-80)
    with method='xcorr' over two files: per file TimeLapseImaging's preprocessing (:50-71, method 'xcorr': no trace
    norm), SurfaceWaveSelector (:166-196), get_images (:198-201: VirtualShotGathersFromWindows, norm=False, no mute),
    then ``avg_image += imagingObj.images.avg_image`` from ``avg_image = 0`` (:39, :67: a sum of per-file means), and
    at the end compute_disp_image() with its defaults and save_avg_disp_to_npz (:199-201, timeLapseImaging.py:205).
    Each file's TimeLapseImaging is a plain object holding the tracking results (the tracker is outside the hot
    path), as in gen_tli."""
    import tempfile

    import apis.timeLapseImaging as tli
    from tests.golden_io import workflow_files
    T = tli.TimeLapseImaging
    out = {}
    avg_image = 0
    for k, c in enumerate(workflow_files()):
        obj = types.SimpleNamespace(method="xcorr", data=c["rec"].copy(), dt=c["t_axis"][1] - c["t_axis"][0],
                                    t_axis=c["t_axis"], x_axis=c["x_axis"],
                                    distances_along_fiber=(c["x_axis"] - 400) * 8.16,
                                    surface_wave_preprecessing_dict=None, start_x=c["start_x_tracking"],
                                    veh_states=c["veh_states"], dist_along_fiber_tracking=c["dist_trk"],
                                    t_axis_tracking=c["t_trk"])
        T._preprocessing_for_surface_waves(obj)
        T.select_surface_wave_windows(obj, c["x0"], **c["select_kw"])
        T.get_images(obj, **c["imaging_kw"])
        out[f"n_windows_{k}"] = np.array(len(obj.sw_selector.windows))
        out[f"w_{k}"] = np.array([im.XCF_out.shape[-1] for im in obj.images.images])
        out[f"file_avg_{k}"] = obj.images.avg_image.XCF_out
        avg_image += obj.images.avg_image
    avg_image.compute_disp_image()
    out.update(day_xcf=avg_image.XCF_out, day_x_axis=avg_image.x_axis, day_t_axis=avg_image.t_axis,
               day_fv=avg_image.disp.fv_map)
    with tempfile.TemporaryDirectory() as d:
        T.save_avg_disp_to_npz(types.SimpleNamespace(images=types.SimpleNamespace(avg_image=avg_image)),
                               fname="day.npz", fdir=d)
        f = np.load(os.path.join(d, "day.npz"), allow_pickle=False)
        out["npz_keys"] = np.array(sorted(f.files))
        assert np.array_equal(f["XCF_out"], avg_image.XCF_out)
    return out


GENERATORS = {"vsg_w500": gen_vsg, "vsg_w499": gen_vsg_w499, "vsg_edge": gen_vsg_edge, "disp": gen_disp,
              "bandpass": gen_bandpass, "ridge": gen_ridge, "fk": gen_fk, "prep": gen_prep, "select": gen_select,
              "tli": gen_tli, "workflow": gen_workflow}


def main(names=None):
    ref = import_reference()
    meta = dict(numpy=np.__version__, scipy=scipy.__version__)
    for name, fn in GENERATORS.items():
        if names and name not in names:
            continue
        out = fn(ref)
        out["meta"] = np.array(repr(meta))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path}: {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":  # python tests/golden/make_golden.py [name ...]
    main(sys.argv[1:])
