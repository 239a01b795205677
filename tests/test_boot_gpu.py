"""GPU parity of the bootstrap path: ridge walk, resample stacks, end-to-end
bootstrap_disp / convergence_test against the reference's goldens (tests/golden/ridge.npz) and the
oracle (oracle/ridge.py)."""
import random

import numpy as np
import pytest
import scipy.interpolate

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
KW = dict(pivot=700, start_x=500, end_x=900)


def _mode1(g):
    return scipy.interpolate.interp1d(g["refvel_f"], g["refvel_v"])


def test_ridge_kernel_matches_reference_goldens(device):
    """dvh_ridge on the reference's own f-v map gives the reference's ridges (walk, reference curve,
    vel_max modes of extract_ridge_ref_idx)."""
    import torch

    from das_diff_veh_amd.bootstrap import ridges
    g = gio.load("ridge")
    fq, vels = g["freqs"], g["vels"]
    fv = torch.as_tensor(g["fv_map"].astype(np.float32), device=device)[None]
    w = ridges(fv, fq, vels, 2.5, 14, ref_freq_idx=80 - int(np.sum(fq < 2.5)), sigma=25, vel_max=800)[0]
    np.testing.assert_allclose(w, g["walk"], rtol=0, atol=1e-9)
    r = ridges(fv, fq, vels, 10, 15, ref_freq_idx=130 - int(np.sum(fq < 10)), sigma=50, vel_max=800,
               ref_vel=_mode1(g))[0]
    np.testing.assert_allclose(r, g["refvel"], rtol=0, atol=1e-9)
    v = ridges(fv, fq, vels, 2.5, 14, sigma=25, vel_max=800)[0]
    np.testing.assert_array_equal(v, g["velmax"])


def test_ridge_negative_reference_index(device):
    """A negative band-relative ref_freq_idx (reachable from bootstrap_disp) is a Python index: the
    reference's pick at column nb + ref and its loop order (golden walk_neg7), and the oracle elsewhere."""
    import torch

    from das_diff_veh_amd.bootstrap import ridges
    from oracle import ridge as orid
    g = gio.load("ridge")
    fq, vels = g["freqs"], g["vels"]
    fv = torch.as_tensor(g["fv_map"].astype(np.float32), device=device)[None]
    m0 = (fq >= 2.5) & (fq < 14)
    np.testing.assert_allclose(ridges(fv, fq, vels, 2.5, 14, ref_freq_idx=-7, sigma=25, vel_max=800)[0],
                               g["walk_neg7"], rtol=0, atol=1e-9)
    nb = int(m0.sum())
    for ref in (-1, -nb):
        o = orid.extract_ridge_ref_idx(fq[m0], vels, g["fv_map"][:, m0], ref_freq_idx=ref, sigma=25, vel_max=800)
        np.testing.assert_allclose(ridges(fv, fq, vels, 2.5, 14, ref_freq_idx=ref, sigma=25, vel_max=800)[0], o,
                                   rtol=0, atol=1e-9)
    with pytest.raises(IndexError):
        ridges(fv, fq, vels, 2.5, 14, ref_freq_idx=-nb - 1, sigma=25, vel_max=800)


@pytest.mark.parametrize("nV", [1000, 63, 65, 1024, 1500])
def test_ridge_velocity_axis_sizes(device, nV):
    """The walk's velocity axis in registers (nV <= 1 024: 16 rows per lane at most, ragged last lane) and the
    global-memory binary search past it: picks (walk, reference-curve and negative-index modes) equal the oracle's
    extract_ridge_ref_idx on a resampled copy of the golden map."""
    import torch

    from das_diff_veh_amd.bootstrap import ridges
    from oracle import ridge as orid
    g = gio.load("ridge")
    fq, vels0, fv0 = g["freqs"], g["vels"], g["fv_map"]
    vels = np.linspace(vels0[0], vels0[-1], nV)  # the golden axis' range and order, nV points
    fvm = fv0[np.linspace(0, vels0.size - 1, nV).round().astype(int)].astype(np.float32)
    fv = torch.as_tensor(fvm, device=device)[None]
    cases = ((2.5, 14, 80 - int(np.sum(fq < 2.5)), 25, None), (2.5, 14, -3, 25, None),
             (10, 15, 130 - int(np.sum(fq < 10)), 50, _mode1(g)))
    for lb, ub, ref, sig, rv in cases:
        m = (fq >= lb) & (fq < ub)
        got = ridges(fv, fq, vels, lb, ub, ref_freq_idx=ref, sigma=sig, vel_max=800, ref_vel=rv)[0]
        want = orid.extract_ridge_ref_idx(fq[m], vels, fvm[:, m].astype(np.float64), ref_freq_idx=ref, sigma=sig,
                                          vel_max=800, ref_vel=rv)
        assert len(got) == int(m.sum())
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-9)


def test_extract_ridge_mirror(device):
    from das_diff_veh_amd.modules.utils import extract_ridge_ref_idx
    g = gio.load("ridge")
    fq, vels, fv = g["freqs"], g["vels"], g["fv_map"]
    m = (fq >= 2.5) & (fq < 14)
    w = extract_ridge_ref_idx(fq[m], vels, fv[:, m], ref_freq_idx=80 - int(np.sum(fq < 2.5)), sigma=25, vel_max=800)
    np.testing.assert_allclose(w, g["walk"], rtol=0, atol=1e-9)
    with pytest.raises(ValueError):  # savgol window longer than the band, as scipy raises
        extract_ridge_ref_idx(fq[:10], vels, fv[:, :10], ref_freq_idx=3)


def _windows():
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    g = gio.load("vsg_w500")
    return [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(gio.n_pass(g))], g


def test_resample_stacks_and_images(device):
    """Resample stacks = mean of the drawn passes' gathers; their f-v images = map_fv of the oracle."""
    from das_diff_veh_amd import bootstrap as bt
    from oracle import disp as odisp
    from oracle import vsg as ovsg
    wins, g = _windows()
    cache = bt.GatherCache(wins, **KW)
    sels = np.array([[1, 3, 4], [2, 2, 1], [4, 1, 2]], dtype=np.int32)
    stacks = cache.resample_stacks(sels).double().cpu().numpy()
    fv = cache.resample_images(sels).cpu().numpy()
    s, e, _ = cache.disp_plan()
    for b, sel in enumerate(sels):
        ref = ovsg.stack([g["xcf"][i] for i in sel])
        assert gio.gather_rel_err(stacks[b], ref[s:e + 1]) < 1e-4
        rfv = odisp.compute_disp_image(ref, g["gather_x_axis"], g["gather_t_axis"], start_x=-150, end_x=0)
        assert np.abs(fv[b] - rfv).max() <= 1e-4 * np.abs(rfv).max()


def test_resample_stacks_sizes_equal_per_size(device):
    """resample_stacks_sizes (convergence's one upload + one dvh_select_mean_var launch) equals resample_stacks
    called per size, row for row, including sizes of one pass, repeated passes and sizes past the kernel's 8-load
    groups, and a float32 sum in selection order divided by the size (sum(images) / len(images)), bit for bit."""
    import torch

    from das_diff_veh_amd import bootstrap as bt
    wins, _ = _windows()
    cache = bt.GatherCache(wins, **KW)
    rng = np.random.default_rng(5)
    sels = [rng.integers(0, cache.n, size=(3, k)).astype(np.int32) for k in (1, 2, 4, 3, 8, 9, 17)]
    got = cache.resample_stacks_sizes(sels)
    want = torch.cat([cache.resample_stacks(x) for x in sels])
    assert torch.equal(got, want)
    s_, e_, _ = cache.disp_plan()
    G = cache.G[:, s_:e_ + 1, :].cpu().numpy()
    ref = []
    for x in sels:
        for row in x:
            acc = np.zeros(G.shape[1:], np.float32)
            for j in row:
                acc += G[j]
            ref.append(acc / np.float32(len(row)))
    assert np.array_equal(got.cpu().numpy(), np.stack(ref))
    with pytest.raises(ValueError):
        cache.resample_stacks_sizes([np.array([[0, cache.n]], np.int32)])


def _walk_audit(dev_picks, ref_picks, ref_fv_band, dev_fv_band, vels, sigma, ref_idx=None, ref_vel=None, fq=None):
    """The ridge walk of extract_ridge_ref_idx (modules/utils.py:621-678) is a masked argmax per column; SURVEY §8(d)'s
    pick rule applied to one step: the device's pick is accepted iff the REFERENCE image attains its maximum over the
    step's window there, ref_fv[pick, i] == max(ref_fv[window, i]), the window being the one the device's walk used
    (around its own previous pick, or the ref_vel band).  Returns, per column in walk order:
      'same'     the device's pick is the reference's;
      'tie'      another index, but the rule holds (an exact float32 tie of the reference image, or a window
                 that an earlier tie moved);
      'near'     the rule fails: (i, device pick, reference value there, reference maximum of the window, the
                 device image's values at both indices) -- a float near-tie the caller reports by these values."""
    vel = np.asarray(vels, dtype=np.float64)[::-1]
    n = len(dev_picks)
    order = list(range(n)) if ref_idx is None else [ref_idx] + list(range(ref_idx - 1, -1, -1)) + list(
        range(ref_idx + 1, n))
    vr = ref_vel(fq) if ref_vel is not None else None
    out = {"same": [], "tie": [], "near": []}
    for i in order:
        if vr is not None:
            mask = (vel > vr[i] - sigma) & (vel < vr[i] + sigma)
        elif i == ref_idx:
            mask = np.ones_like(vel, dtype=bool)
        else:
            prev = dev_picks[i + 1] if i < ref_idx else dev_picks[i - 1]
            mask = (vel > prev - sigma) & (vel < prev + sigma)
        col = ref_fv_band[:, i]
        d = int(np.flatnonzero(vel == dev_picks[i])[0])
        r = int(np.flatnonzero(vel == ref_picks[i])[0])
        assert mask[d], (i, "device pick outside its own window")
        if d == r:
            out["same"].append(i)
        elif col[d] == col[mask].max():
            out["tie"].append(i)
        else:
            rm = int(np.flatnonzero(mask)[np.argmax(col[mask])])
            out["near"].append((i, float(dev_picks[i]), float(col[d]), float(col[rm]), float(dev_fv_band[d, i]),
                                float(dev_fv_band[rm, i])))
    return out


def _audit_report(name, audits, fv_err):
    """Asserts the near-tie steps are float near-ties of the two images: the reference prefers its maximum by
    less than the images' measured discrepancy, and the device image prefers its pick by less than it too."""
    near = [x for a in audits for x in a["near"]]
    ties = sum(len(a["tie"]) for a in audits)
    for i, v, ref_at, ref_max, dev_at, dev_max in near:
        print(f"{name}: column {i}: device {v} m/s, reference image {ref_at!r} vs its window maximum {ref_max!r} "
              f"(gap {ref_max - ref_at:.3e}); device image {dev_at!r} vs {dev_max!r} (gap {dev_at - dev_max:.3e}); "
              f"measured f-v discrepancy {fv_err:.3e}")
        assert 0 < ref_max - ref_at <= 2 * fv_err and 0 <= dev_at - dev_max <= 2 * fv_err
    print(f"{name}: {sum(len(a['same']) for a in audits)} picks equal, {ties} exact ties / tie-moved windows "
          f"(SURVEY 8(d) rule holds), {len(near)} float near-ties")
    return len(near)


def _image_picks_rule(dev_fv, ref_fv):
    """SURVEY §8(d) on a whole f-v image: every column's argmax of the device image attains the reference maximum."""
    from oracle import disp as odisp
    ok = odisp.pick_ok(ref_fv, np.asarray(dev_fv).argmax(axis=0))
    assert np.all(ok), f"{(~ok).sum()} of {ok.size} image picks miss the reference maximum"


def test_bootstrap_disp_matches_reference(device):
    """Same draws as the reference (random.seed).  Per resample: the image's picks meet SURVEY §8(d) against the
    reference's own f-v map (tests/golden/ridge.npz:boot_fv); per resample and mode, the ridge walk on our images
    equals the oracle's walk on the same images (1e-9), and every step of it is audited against the reference's
    image under §8(d) (_walk_audit): equal picks, exact ties, or float near-ties reported by both images' values;
    with identical picks the smoothed ridges equal the reference's to 1e-9."""
    from das_diff_veh_amd import bootstrap as bt
    from das_diff_veh_amd.apis.imaging_classes import bootstrap_disp
    from oracle import ridge as orid
    wins, _ = _windows()
    g = gio.load("ridge")
    mode1 = _mode1(g)
    random.seed(11)
    rv, fq = bootstrap_disp(wins, 3, 4, [25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    np.testing.assert_array_equal(fq, g["boot_freqs"])
    random.seed(11)
    sels = bt.draw(len(wins), 3, 4)
    np.testing.assert_array_equal(sels, g["boot_sel"])
    cache = bt.GatherCache(wins, **KW)
    fv_dev = cache.resample_images(sels)
    fv = fv_dev.cpu().numpy()
    audits, fv_err = [], 0.0
    for b in range(4):
        ref_fv = g["boot_fv"][b]
        err = np.abs(fv[b].astype(np.float64) - ref_fv).max()
        assert err <= 1e-4 * np.abs(ref_fv).max()
        fv_err = max(fv_err, float(err))
        _image_picks_rule(fv[b], ref_fv)
        for m, (lb, ub, ri, sg, vr, key) in enumerate(((2.5, 14, 80, 25, None, "boot_mode0"),
                                                       (10, 15, 130, 50, mode1, "boot_mode1"))):
            band = (fq >= lb) & (fq < ub)
            ref_idx = ri - int(np.sum(fq < lb))
            # the walk's logic: device walk == oracle walk on our own image
            o = orid.extract_ridge_ref_idx(fq[band], bt.VELS, fv[b][:, band], ref_freq_idx=ref_idx, sigma=sg,
                                           vel_max=800, ref_vel=vr)
            np.testing.assert_allclose(rv[m][b], o, rtol=0, atol=1e-9)
            # the picks: device (on our image) vs reference (on the reference's image)
            _, dp = bt.ridges(fv_dev[b:b + 1], fq, bt.VELS, lb, ub, ref_freq_idx=ref_idx, sigma=sg, vel_max=800,
                              ref_vel=vr, return_picks=True)
            _, rp = orid.extract_ridge_ref_idx(fq[band], bt.VELS, ref_fv[:, band], ref_freq_idx=ref_idx, sigma=sg,
                                               vel_max=800, ref_vel=vr, return_picks=True)
            a = _walk_audit(dp[0], rp, ref_fv[:, band], fv[b][:, band], bt.VELS, sg, ref_idx=None if vr is not None else ref_idx,
                            ref_vel=vr, fq=fq[band])
            audits.append(a)
            if not a["tie"] and not a["near"]:
                np.testing.assert_allclose(rv[m][b], g[key][b], rtol=0, atol=1e-9)
    n_near = _audit_report("bootstrap_disp", audits, fv_err)
    assert n_near <= 2, n_near


def test_convergence_test_small(device):
    """convergence_test (imaging_diff_speed.ipynb#cell30) for bt_size 1..3: each entry equals the summed std of the
    device ridges of the same draws (1e-9); every resample image's picks meet SURVEY §8(d) against the reference-
    pinned oracle's image (f64 VSG + map_fv), and every walk step is audited under §8(d) (_walk_audit); where a
    (bt_size, mode) has no differing pick the entry equals the oracle's to 1e-9."""
    from das_diff_veh_amd import bootstrap as bt
    from das_diff_veh_amd.apis.imaging_classes import convergence_test
    from oracle import disp as odisp
    from oracle import ridge as orid
    from oracle import vsg as ovsg
    wins, g5 = _windows()
    g = gio.load("ridge")
    mode1 = _mode1(g)
    modes = ((2.5, 14, 80, 25, None), (10, 15, 130, 50, mode1))
    args = ([25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    random.seed(5)
    got = convergence_test(3, wins, 4, *args)
    random.seed(5)
    ow = [gio.oracle_window(g5, i) for i in range(len(wins))]
    og = [ovsg.virtual_shot_gather(w, include_other_side=True, norm=False, **KW, wlen=2) for w in ow]
    cache = bt.GatherCache(wins, **KW)
    fq = bt.FREQS
    audits, fv_err = [], 0.0
    for k in range(1, 4):
        sels = bt.draw(len(wins), k, 4)
        fv_dev = cache.resample_images(sels)
        fv_np = fv_dev.cpu().numpy()
        ref_fv = [odisp.compute_disp_image(ovsg.stack([og[i][0] for i in sel]), og[0][1], og[0][2], start_x=-150,
                                           end_x=0) for sel in sels]
        for b in range(4):
            fv_err = max(fv_err, float(np.abs(fv_np[b].astype(np.float64) - ref_fv[b]).max()))
            _image_picks_rule(fv_np[b], ref_fv[b])
        for m, (lb, ub, ri, sg, vr) in enumerate(modes):
            band = (fq >= lb) & (fq < ub)
            ref_idx = ri - int(np.sum(fq < lb))
            sm, dp = bt.ridges(fv_dev, fq, bt.VELS, lb, ub, ref_freq_idx=ref_idx, sigma=sg, vel_max=800, ref_vel=vr,
                               return_picks=True)
            assert abs(np.sum(np.std(sm, axis=0)) - got[m, k - 1]) <= 1e-9
            differ, ref_sm = 0, []
            for b in range(4):
                r, rp = orid.extract_ridge_ref_idx(fq[band], bt.VELS, ref_fv[b][:, band], ref_freq_idx=ref_idx,
                                                   sigma=sg, vel_max=800, ref_vel=vr, return_picks=True)
                a = _walk_audit(dp[b], rp, ref_fv[b][:, band], fv_np[b][:, band], bt.VELS, sg,
                                ref_idx=None if vr is not None else ref_idx, ref_vel=vr, fq=fq[band])
                audits.append(a)
                differ += len(a["tie"]) + len(a["near"])
                ref_sm.append(r)
            if not differ:
                assert abs(np.sum(np.std(np.stack(ref_sm), axis=0)) - got[m, k - 1]) <= 1e-9
    n_near = _audit_report("convergence_test", audits, fv_err)
    assert n_near <= 4, n_near


def _mixed_windows():
    """The w = 500 and w = 499 fixtures' passes interleaved (one 56 x 4 096 shape): real records mix both lag lengths
    (int(wlen / dt) of each window's own time step, apis/virtual_shot_gather.py:18,41)."""
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    g5, g9 = gio.load("vsg_w500"), gio.load("vsg_w499")
    srcs = [(g5, 0), (g9, 0), (g5, 1), (g5, 2), (g9, 1), (g5, 3), (g5, 4)]
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for g, i in srcs]
    ow = [gio.oracle_window(g, i) for g, i in srcs]
    return wins, ow


def test_mixed_lag_lengths_resample_images(device):
    """A gather cache over windows of w = 500 and 499: each resample's stack is the reference's sum(images) on its
    first drawn pass's lag axis (VirtualShotGather.__add__ truncating the others, apis/virtual_shot_gather.py:195-199)
    and its f-v image is compute_disp_image on that axis -- against the oracle (oracle.vsg.stack, oracle.disp), for
    draws led by either length, within 1e-4, picks on the reference maximum."""
    from das_diff_veh_amd import bootstrap as bt
    from oracle import disp as odisp
    from oracle import vsg as ovsg
    wins, ow = _mixed_windows()
    og = [ovsg.virtual_shot_gather(w, include_other_side=True, norm=False, **KW, wlen=2) for w in ow]
    assert {x[0].shape[-1] for x in og} == {499, 500}
    cache = bt.GatherCache(wins, **KW)
    sels = np.array([[1, 2, 3], [2, 1, 4], [4, 6, 1], [3, 5, 2], [6, 1, 1]], dtype=np.int32)
    fv = cache.resample_images(sels).cpu().numpy()
    for b, sel in enumerate(sels):
        ref = ovsg.stack([og[i][0] for i in sel])
        rfv = odisp.compute_disp_image(ref, og[sel[0]][1], og[sel[0]][2], start_x=-150, end_x=0)
        assert np.abs(fv[b] - rfv).max() <= 1e-4 * np.abs(rfv).max(), b
        _image_picks_rule(fv[b], rfv)


def test_mixed_lag_lengths_bootstrap_and_convergence(device):
    """bootstrap_disp and convergence_test over the mixed windows: the reference's draws (random.seed), every
    resample's ridges equal the walk of the oracle on our own images (1e-9), and the images match the oracle's."""
    from das_diff_veh_amd import bootstrap as bt
    from das_diff_veh_amd.apis.imaging_classes import bootstrap_disp, convergence_test
    from oracle import ridge as orid
    wins, ow = _mixed_windows()
    g = gio.load("ridge")
    mode1 = _mode1(g)
    args = ([25, 50], 700, 500, 900, [80, 130], [2.5, 10], [14, 15], [None, mode1])
    random.seed(4)  # draws led by w = 500 and by w = 499 passes
    rv, fq = bootstrap_disp(wins, 3, 6, *args)
    random.seed(4)
    sels = bt.draw(len(wins), 3, 6)
    assert len({int(bt.GatherCache(wins, **KW).w_of[s[0]]) for s in sels}) == 2  # draws led by both lengths
    fv = bt.GatherCache(wins, **KW).resample_images(sels).cpu().numpy()
    for b in range(6):
        for m, (lb, ub, ri, sg, vr) in enumerate(((2.5, 14, 80, 25, None), (10, 15, 130, 50, mode1))):
            band = (fq >= lb) & (fq < ub)
            o = orid.extract_ridge_ref_idx(fq[band], bt.VELS, fv[b][:, band], ref_freq_idx=ri - int(np.sum(fq < lb)),
                                           sigma=sg, vel_max=800, ref_vel=vr)
            np.testing.assert_allclose(rv[m][b], o, rtol=0, atol=1e-9)
    random.seed(5)
    got = convergence_test(2, wins, 3, *args)
    assert got.shape == (2, 2) and np.all(np.isfinite(got))
