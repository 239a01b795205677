"""Host-side logic (no GPU): index tables, the C-ABI library, schedules, dispersion tables."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.interpolate
import scipy.signal

from tests import golden_io as gio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_interp1d_matches_scipy_bitwise():
    from das_diff_veh_amd.plan import interp1d_extrap
    rng = np.random.default_rng(0)
    x = np.sort(rng.uniform(0, 1000, 200))
    x = x[np.r_[True, np.diff(x) > 0]]
    y = 3.0 + x / 17.3 + rng.normal(0, 0.01, x.size)
    q = np.concatenate([rng.uniform(-100, 1100, 500), x[:10]])
    ref = scipy.interpolate.interp1d(x[::-1], y[::-1], fill_value="extrapolate")(q)
    assert np.array_equal(interp1d_extrap(x[::-1], y[::-1])(q), ref)


def test_py_slice_semantics():
    from das_diff_veh_amd.plan import py_slice
    n = 17
    for a in range(-25, 25):
        for b in range(-25, 25):
            s, L = py_slice(a, b, n)
            ref = np.arange(n)[a:b]
            assert L == ref.size and (L == 0 or s == ref[0])


def test_first_true_ge():
    from das_diff_veh_amd.plan import first_true_ge
    t = 4.0 + np.arange(100) * 0.004
    q = np.array([-1.0, 4.0, 4.0041, 4.396, 4.3961, 100.0, np.nan])
    ref = np.array([np.argmax(t >= v) for v in q])
    assert np.array_equal(first_true_ge(t, q), ref)


@pytest.mark.parametrize("fixture", ["vsg_w500", "vsg_w499"])
def test_plan_matches_oracle_slices(fixture):
    """Every (start, length) the kernels will read is the slice the reference takes."""
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.plan import VsgParams, pass_geometry
    g = gio.load(fixture)
    prm = VsgParams(pivot=700, start_x=500, end_x=900, include_other_side=True, norm=False)
    for i in range(gio.n_pass(g)):
        w = SurfaceWaveWindow(**gio.pass_arrays(g, i))
        geo = pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, prm)
        f = scipy.interpolate.interp1d(w.veh_state_x, w.veh_state_t, fill_value="extrapolate")
        T = w.t_axis.size
        for side, sgn in ((0, 1), (1, -1)):
            pt = int(np.argmax(w.t_axis >= f(700) + sgn * 1))
            for r in range(geo.start_idx, geo.end_idx):
                shared = r <= geo.pivot_idx if sgn > 0 else r >= geo.pivot_idx
                if shared:
                    sl = slice(pt, pt + geo.nsamp) if sgn > 0 else slice(pt - geo.nsamp, pt)
                else:
                    ti = int(np.argmax(w.t_axis >= f(w.x_axis[r]) + sgn * 1))
                    sl = slice(ti, ti + geo.nsamp) if sgn > 0 else slice(ti - geo.nsamp, ti)
                idx = np.arange(T)[sl]
                a, L = geo.seg[r - geo.start_idx, side]
                assert L == idx.size and (L == 0 or a == idx[0]), (i, side, r)


def test_plan_rejects_dt_004():
    from das_diff_veh_amd.plan import VsgParams, pass_geometry
    t = np.arange(1000) * 0.004
    with pytest.raises(ValueError):
        pass_geometry(np.arange(60) * 8.16 + 460, t, np.arange(300.0, 1000.0), np.linspace(0, 4, 700),
                      VsgParams(pivot=700, start_x=500, end_x=900))


def test_stack_schedule():
    from das_diff_veh_amd.vsg import StackSchedule
    slots = np.array([2, 0, 1, 1, 0, 2, 2, 2, 1, 0, 0])
    s = StackSchedule(slots, 3, chunk=2)
    seen = np.zeros(slots.size, int)
    for b, e, slot in s.chunk_tab:
        assert e - b <= 2
        for q in range(b, e):
            assert slots[s.order[q]] == slot
            seen[s.order[q]] += 1
    assert (seen == 1).all()
    np.testing.assert_allclose(s.weights, 1.0 / np.bincount(slots)[slots])


def test_savgol_operator_matches_scipy():
    from das_diff_veh_amd.disp import savgol_operator
    rng = np.random.default_rng(1)
    x = rng.standard_normal(242).astype(np.float32)
    h, el, er = savgol_operator(25, 4)
    y = np.empty(242)
    for f in range(242):
        if f < 12:
            y[f] = el[f] @ x[:25]
        elif f >= 230:
            y[f] = er[f - 230] @ x[-25:]
        else:
            y[f] = h @ x[f - 12:f + 13]
    ref = scipy.signal.savgol_filter(x, 25, 4)
    assert np.abs(y - ref).max() < 1e-5


def test_disp_plan_reproduces_reference_bilinear_on_host():
    """The host tables + kernel formula (evaluated here in numpy) give the oracle's f-v map."""
    from das_diff_veh_amd.disp import DispPlan
    from oracle import disp as odisp
    g = gio.load("vsg_w500")
    s = np.abs(g["gather_x_axis"] + 200).argmin()
    e = np.abs(g["gather_x_axis"] - 0).argmin()
    data = g["stack"][s:e + 1]
    dt = g["gather_t_axis"][1] - g["gather_t_axis"][0]
    freqs, vels = np.arange(0.8, 25, 0.1), np.arange(200, 1200)
    p = DispPlan(data.shape[0], data.shape[1], 8.16, dt, freqs, vels)
    res, _, _ = odisp.fk(data, 8.16, dt)
    fk = res[p.m_lo:p.m_lo + p.n_kb, p.j_lo:p.j_lo + p.n_fb]
    # the twiddle tables reproduce the full fft2 on the compact grid
    D = data @ (p.wt[:, 0::2] + 1j * p.wt[:, 1::2])
    Z = (p.atab[:p.n_kb, :data.shape[0]] + 1j * p.atab[p.MT:p.MT + p.n_kb, :data.shape[0]]) @ D
    np.testing.assert_allclose(np.abs(Z), fk, rtol=1e-9, atol=1e-9 * fk.max())
    raw = np.empty((p.nF, p.nV))
    for f in range(p.nF):
        q = np.clip(p.kq[f], p.kmin, p.kmax)
        m = np.clip(np.searchsorted(p.kgrid, q, side="right") - 1, 0, p.n_kb - 2)
        klo, khi = p.kgrid[m], p.kgrid[m + 1]
        fx = 1.0 / (khi - klo)
        hx0, hx1 = fx * (khi - q), fx * (q - klo)
        j = p.fj[f]
        hy0, hy1 = p.fw[f]
        raw[f] = fk[m, j] * hx0 * hy0 + fk[m, j + 1] * hx0 * hy1 + fk[m + 1, j] * hx1 * hy0 + \
            fk[m + 1, j + 1] * hx1 * hy1
    fv = scipy.signal.savgol_filter(raw.astype(np.float32), 25, 4, axis=0).T
    assert np.abs(fv - g["fv_map"]).max() <= 1e-6 * np.abs(g["fv_map"]).max()


def test_library_exports_every_header_symbol():
    """libdvh.so loads without a GPU and exports every entry point include/dvh.h declares."""
    from das_diff_veh_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from das_diff_veh_amd.build import build
        build()
    hdr = open(os.path.join(ROOT, "include", "dvh.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(dvh_\w+)\(", hdr, flags=re.M))
    assert len(declared) >= 14
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    assert _lib.load().dvh_abi_version() == 2
    assert _lib.load().dvh_vsg_fft_length(500) == 500
    assert _lib.load().dvh_vsg_fft_length(499) == 1024
    assert _lib.load().dvh_vsg_fft_length(5000) == 0


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.apis.virtual_shot_gather import VirtualShotGather
    g = gio.load("vsg_w500")
    w = SurfaceWaveWindow(**gio.pass_arrays(g, 0))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        VirtualShotGather(w, include_other_side=True, pivot=700, start_x=500, end_x=900)


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "das_diff_veh_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f


@pytest.mark.parametrize("case", ["default", "short", "odd", "spacing"])
def test_pass_table_matches_reference(case):
    """select.pass_table (host index bookkeeping of locate_windows) vs the reference's windows."""
    from das_diff_veh_amd.plan import py_slice
    from das_diff_veh_amd.select import pass_table
    g = gio.load("select")
    c = gio.select_cases()[case]
    t_axis = c["t_axis"]
    ks, (sx, ex), t0, t1 = pass_table(t_axis, c["dist"], c["x0"], c["start_x_tracking"], c["veh_states"], c["t_trk"],
                                      t_axis[1] - t_axis[0], **c["kw"])
    a, n = py_slice(t0, t1, c["rec"].shape[1])
    got = np.stack([ks, np.full_like(ks, sx), np.full_like(ks, ex), a, a + n], axis=1) if ks.size else \
        np.zeros((0, 5), np.int64)
    assert np.array_equal(got, g[case + "_windows"])


def test_pass_table_untracked_crossing_raises():
    """int(nan) in locate_windows raises ValueError; so does the host table."""
    from das_diff_veh_amd.select import pass_table
    c = gio.select_cases()["short"]
    vs = c["veh_states"].copy()
    vs[2, c["x0"] - c["start_x_tracking"]] = np.nan
    with pytest.raises(ValueError):
        pass_table(c["t_axis"], c["dist"], c["x0"], c["start_x_tracking"], vs, c["t_trk"], 0.004, wlen_sw=2)


def _sliding_case(n_ch=300, n_t=8192, seed=5):
    from das_diff_veh_amd.synth import TRACK_DT, DT_W500
    rng = np.random.default_rng(seed)
    x_axis = 0.37 + 8.16 * np.arange(n_ch)
    t_axis = DT_W500 + np.arange(n_t) * 0.004
    trk = []
    for _ in range(4):
        x0, v = rng.uniform(600, 1800), rng.uniform(15, 30)
        tc = t_axis[n_t // 2] + rng.uniform(-1, 1)
        xs = np.arange(np.floor(x0) - 1500, np.floor(x0) + 1500, 1.0)
        trk.append((xs, np.round((tc + (xs - x0) / v) / TRACK_DT) * TRACK_DT))
    return x_axis, t_axis, trk


def test_sliding_geometry_matches_pass_geometry():
    """Vectorised sliding-pivot tables == pass_geometry at each pivot (start_x / end_x = pivot -/+ 200)."""
    from das_diff_veh_amd.plan import (UnitPlan, VsgParams, pass_geometry, sliding_full, sliding_geometry,
                                       sliding_pivots)
    x_axis, t_axis, trk = _sliding_case()
    pch = np.arange(32, 300 - 32, 8)
    prm = VsgParams(include_other_side=True, norm=False)
    spatial = sliding_pivots(x_axis, pch, 200.0)
    n_full = 0
    for vx, vt in trk:
        seg, full = sliding_geometry(x_axis, t_axis, vx, vt, spatial, prm)
        assert np.array_equal(full, sliding_full(x_axis, t_axis, vx, vt, spatial, prm))
        n_full += int(full.sum())
        for j, c in enumerate(pch):
            p = float(x_axis[c])
            g = pass_geometry(x_axis, t_axis, vx, vt, VsgParams(pivot=p, start_x=p - 200.0, end_x=p + 200.0,
                                                                  include_other_side=True, norm=False))
            assert (g.pivot_idx, g.start_idx, g.end_idx) == (spatial[0][j], spatial[1][j], spatial[2][j])
            assert np.array_equal(g.seg, seg[j]), j
            assert full[j] == bool(np.all(g.seg[:, :, 1] == g.nsamp))
    assert n_full > 0
    plan = UnitPlan.sliding(x_axis, t_axis, trk, pch, 200.0, prm)
    assert plan.n_pass == n_full and plan.R == 49
    # unit u reads window q's channels at q * C + c of the flattened record
    q, j = plan.unit_window[3], plan.unit_pivot[3]
    assert plan.pass_tab[3, 1] == q * 300 + spatial[0][j]


def test_algorithmic_bytes_union_matches_loop():
    """seg_algorithmic_bytes' vectorised pivot-interval union equals a plain interval merge."""
    from das_diff_veh_amd.plan import seg_algorithmic_bytes, seg_nwin
    rng = np.random.default_rng(3)
    seg = np.zeros((7, 13, 2, 2), dtype=np.int64)
    seg[..., 0] = rng.integers(0, 3000, seg.shape[:3])
    seg[..., 1] = rng.choice([0, 400, 500, 999, 1000], seg.shape[:3])
    w, hop = 500, 250
    for sides in (1, 2):
        nw = seg_nwin(seg, w, hop)[:, :, :sides]
        cov = np.where(nw > 0, (nw - 1) * hop + w, 0)
        piv = 0
        for p in range(seg.shape[0]):
            covered = np.zeros(5000, bool)
            for a, c in zip(seg[p, :, :sides, 0].ravel(), cov[p].ravel()):
                covered[a:a + c] = True
            piv += 4 * int(covered.sum())
        assert seg_algorithmic_bytes(seg, w, hop, sides, 2) == 4 * int(cov.sum()) + piv + 4 * 2 * w


def test_ridge_npz_writer(tmp_path):
    """save_ridge_npz: the notebook's data/<x0>_speeds.npz keys (imaging_diff_speed.ipynb#cell27), pickle-free
    by default, or the ragged object-array layout the notebook itself writes."""
    from das_diff_veh_amd.bootstrap import load_ridge_npz, save_ridge_npz
    fq = np.arange(0.8, 25, 0.1)
    rv = [[np.arange(116.0) + i for i in range(4)], [np.arange(50.0) - i for i in range(4)]]
    p = tmp_path / "700_speeds.npz"
    save_ridge_npz(p, fq, [2.5, 10], [14, 15], fast=rv, slow=rv)
    f, lb, ub, r = load_ridge_npz(p)
    assert np.array_equal(f, fq) and list(lb) == [2.5, 10] and list(ub) == [14, 15]
    assert set(r) == {"fast", "slow"} and r["fast"][0].shape == (4, 116) and r["fast"][1].shape == (4, 50)
    assert np.array_equal(r["slow"][1][3], rv[1][3])
    q = tmp_path / "700_ref_layout.npz"
    save_ridge_npz(q, fq, [2.5, 10], [14, 15], reference_layout=True, fast=rv)
    with np.load(q, allow_pickle=False) as z:
        assert set(z.files) == {"freqs", "freq_lb", "freq_ub", "vels_fast"}
        with pytest.raises(ValueError):  # the object array needs the notebook's allow_pickle=True
            z["vels_fast"]


def _failing_windows():
    """Golden passes 0 and 3 plus three that cannot be imaged: a one-point trajectory, a gather geometry
    the pivot falls outside of, and dt = 0.004 (the reference's window-length ValueError)."""
    import copy

    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    g = gio.load("vsg_w500")
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(5)]
    trk = copy.copy(wins[1])
    trk.veh_state_x, trk.veh_state_t = trk.veh_state_x[:1], trk.veh_state_t[:1]
    geo = copy.copy(wins[2])
    geo.x_axis = wins[2].x_axis + 1000.0
    d4 = copy.copy(wins[4])
    d4.t_axis = np.arange(wins[4].t_axis.size) * 0.004
    return [wins[0], trk, geo, d4, wins[3]], g


def test_pass_failures_skip_and_count():
    """a failure status per pass (skip + count), decided on the host before any launch."""
    from das_diff_veh_amd.engine import pass_failures
    from das_diff_veh_amd.plan import VsgParams
    wins, _ = _failing_windows()
    prm = VsgParams(pivot=700, start_x=500, end_x=900, include_other_side=True, norm=False)
    failed, axes = pass_failures(wins, prm)
    assert sorted(failed) == [1, 2, 3], failed
    assert "trajectory" in failed[1] and "geometry" in failed[2] and "broadcast" in failed[3]
    assert axes[0] is not None and axes[4] is not None and axes[1] is None


def test_unit_plan_concat():
    """UnitPlan.concat: one launch's tables over several trajectory batches on the same windows."""
    from das_diff_veh_amd.plan import UnitPlan, VsgParams
    x = 0.37 * 8.16 + 8.16 * np.arange(300)
    t = 0.003999999999997783 * np.arange(8192)
    rng = np.random.default_rng(3)

    def trks(n):
        out = []
        for xa, va in zip(rng.uniform(x[40], x[-40], n), rng.uniform(15, 30, n)):
            xs = np.arange(np.floor(xa) - 800.0, np.floor(xa) + 801.0)
            out.append((xs, np.round((t[4096] + (xs - xa) / va) / 0.02) * 0.02))
        return out
    prm = VsgParams(wlen=2, norm=False, include_other_side=True)
    pch = np.arange(32, 268, 8)
    a = UnitPlan.sliding(x, t, trks(3), pch, 200.0, prm)
    b = UnitPlan.sliding(x, t, trks(3), pch, 200.0, prm)
    c = UnitPlan.concat([a, b])
    assert c.n_pass == a.n_pass + b.n_pass
    assert np.array_equal(c.seg_tab, np.concatenate([a.seg_tab, b.seg_tab]))
    assert np.array_equal(c.pass_tab, np.concatenate([a.pass_tab, b.pass_tab]))
    assert np.array_equal(c.unit_window, np.concatenate([a.unit_window, b.unit_window]))
    other = UnitPlan.sliding(x, t, trks(2), pch[:-1], 200.0, prm)
    with pytest.raises(ValueError):
        UnitPlan.concat([a, other])


@pytest.mark.parametrize("nv,nf", [(1000, 242), (512, 1000)])
def test_fv_cell_tables_address_every_stencil_cell(nv, nf):
    """DispPlan.cell_tables (dvh_disp_fv_cells): for every block and every (f, v) it samples, the compact
    indices reach exactly FK[m, j], FK[m + 1, j], FK[m, j + 1], FK[m + 1, j + 1] of the plan's own FITPACK
    intervals, through the block's staged cells only."""
    from das_diff_veh_amd.disp import DispPlan
    dt = 0.003999999999997783
    freqs = np.arange(0.8, 25, 0.1) if nf == 242 else np.linspace(1.0, 24.0, nf)
    vels = np.arange(200, 200 + nv) if nv == 1000 else np.linspace(150.0, 1200.0, nv)
    plan = DispPlan(25, 500, 8.16, dt, freqs, vels)
    ct = plan.cell_tables()
    assert ct is not None
    T, VT, pad = DispPlan.TILE_THREADS, DispPlan.TILE_VT, DispPlan.TILE_PAD
    rng = np.random.default_rng(0)
    FK = rng.standard_normal((plan.n_kb, plan.n_fb))
    flat = FK.ravel()
    nt, TO = ct["n_tile"], ct["TO"]
    nvc = -(-plan.nV // VT)
    assert ct["cell_off"].shape == (nvc * nt, ct["max_cell"])
    for c in range(nvc):
        vs = np.arange(c * VT, min(plan.nV, c * VT + VT))
        for t in range(nt):
            k = c * nt + t
            cells = flat[ct["cell_off"][k, :ct["n_cell"][k]]]
            f_lo, f_hi = t * TO, min(plan.nF, t * TO + TO)
            s0, s1 = max(0, f_lo - pad), min(plan.nF, max(f_hi + pad, plan.sgl))
            assert s1 - s0 <= T
            q = ct["qidx"][k, :s1 - s0, :vs.size]
            m = plan.mk[s0:s1, vs]
            j = plan.fj[s0:s1, None]
            assert np.array_equal(q[..., 2], m)
            assert np.array_equal(cells[q[..., 0]], FK[m, j]) and np.array_equal(cells[q[..., 0] + 1], FK[m + 1, j])
            assert np.array_equal(cells[q[..., 1]], FK[m, j + 1]) and np.array_equal(cells[q[..., 1] + 1], FK[m + 1, j + 1])
    # the point of the tables: a block stages a few rows per column, not the n_kb rows
    assert ct["max_cell"] < 0.5 * plan.n_kb * plan.n_fb
    print("cells per block", int(ct["n_cell"].mean()), "of", plan.n_kb * plan.n_fb)


@pytest.mark.parametrize("nv,nf", [(1000, 242), (512, 1000), (61, 33)])
def test_fv_mfma_tables_reproduce_interp2d(nv, nf):
    """DispPlan.mfma_tables (dvh_disp_fv_mfma): the per-(f, v) FITPACK weights hx and compact cell offsets
    cb, combined the way the kernel does (z00 hx0 hy0 + z01 hx0 hy1 + z10 hx1 hy0 + z11 hx1 hy1), give the
    oracle's interp2d bilinear samples (oracle/disp.py bilinear, modules/utils.py:466-472) on a random
    full FK grid to float64 rounding, and the weights are those of the plan's own intervals."""
    from das_diff_veh_amd.disp import DispPlan
    from oracle import disp as odisp
    dt = 0.003999999999997783
    freqs = np.arange(0.8, 25, 0.1) if nf == 242 else np.linspace(1.0, 24.0, nf)
    vels = np.arange(200, 200 + nv) if nv == 1000 else np.linspace(150.0, 1200.0, nv)
    plan = DispPlan(25, 500, 8.16, dt, freqs, vels)
    mt = plan.mfma_tables()
    hx, cb = mt["hx"], mt["cb"]
    assert hx.shape == (plan.nF, plan.nV, 2) and hx.dtype == np.float64
    assert cb.shape == (plan.nF, plan.nV) and cb.dtype == np.int32
    rng = np.random.default_rng(1)
    res = rng.random((plan.nk, plan.nf))
    comp = res[plan.m_lo:plan.m_lo + plan.n_kb, plan.j_lo:plan.j_lo + plan.n_fb].ravel()
    for f in range(0, plan.nF, max(1, plan.nF // 17)):
        base = cb[f]
        hy0, hy1 = plan.fw[f]
        got = (comp[base] * hx[f, :, 0] * hy0 + comp[base + 1] * hx[f, :, 0] * hy1
               + comp[base + plan.n_fb] * hx[f, :, 1] * hy0 + comp[base + plan.n_fb + 1] * hx[f, :, 1] * hy1)
        ref = odisp.bilinear(res, plan.fft_f, plan.fft_k, np.divide(np.ones(plan.nV) * plan.freqs[f], plan.vels),
                             plan.freqs[f])
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max(), f
    assert np.array_equal(cb // plan.n_fb, plan.mk)
    assert np.all(cb % plan.n_fb == plan.fj[:, None])


def test_native_draws_equal_python_random_sample():
    """bootstrap.draw forms random.sample(range(1, n), k) draws in the library (dvh_random_sample) from the
    generator's Mersenne Twister state: bit-identical to Python's own calls for the set (n > setsize) and pool
    (small n) branches, k = 0 .. 60, and the generator continues exactly where Python's calls leave it."""
    import random

    from das_diff_veh_amd import bootstrap as bt
    for n, ks, times in ((1442, range(0, 61), 30), (7, range(0, 7), 5), (30, (1, 5, 6, 20, 29), 4),
                         (100, (6, 33, 99), 3), (2, (0, 1), 4)):
        for k in ks:
            ra, rb = random.Random(1234 + n + k), random.Random(1234 + n + k)
            got = bt.draw(n, k, times, rand=ra)
            ref = np.array([rb.sample(range(1, n), k) for _ in range(times)], dtype=np.int32).reshape(times, k)
            assert np.array_equal(got, ref), (n, k)
            assert ra.random() == rb.random() and ra.getrandbits(64) == rb.getrandbits(64), (n, k)
    # the module-level generator (the reference's random.seed / random.sample)
    random.seed(7)
    got = bt.draw(1442, 60, 30)
    random.seed(7)
    ref = np.array([random.sample(range(1, 1442), 60) for _ in range(30)], dtype=np.int32)
    assert np.array_equal(got, ref)
    with pytest.raises(ValueError):
        bt.draw(5, 5, 1)


def test_host_gather_packs_windows():
    """dvh_host_gather (device.py's staging copy, host only): n windows packed back to back, any alignment."""
    from das_diff_veh_amd import _lib
    rng = np.random.default_rng(3)
    hs = [rng.standard_normal((7, 131)).astype(np.float32) for _ in range(9)]
    per = hs[0].nbytes
    srcs = (ctypes.c_void_p * len(hs))(*[h.ctypes.data for h in hs])
    for off in (0, 4, 12):
        dst = np.zeros(len(hs) * per + 16, np.uint8)
        _lib.call("dvh_host_gather", ctypes.c_void_p(dst.ctypes.data + off), ctypes.byref(srcs, 8), per, len(hs) - 1)
        got = dst[off:off + (len(hs) - 1) * per].view(np.float32).reshape(len(hs) - 1, 7, 131)
        assert all(np.array_equal(got[j], hs[j + 1]) for j in range(len(hs) - 1))
        assert not dst[off + (len(hs) - 1) * per:].any() and not dst[:off].any()
    assert _lib.load().dvh_host_gather(None, None, per, 1) != 0


def test_rows_of_staged_batch():
    """engine._rows_of: a group's rows of the early-staged batch (evaluated once), the batch itself when the group
    is every window in order; engine._OwnAxes: each pass owns its axes, copied on first access."""
    import torch

    from das_diff_veh_amd import engine
    calls = []

    def batch():
        calls.append(1)
        return torch.arange(12.0).view(6, 2)
    memo = {}
    whole = engine._rows_of(batch, range(6), 6, memo)()
    part = engine._rows_of(batch, [1, 3, 5], 6, memo)()
    assert len(calls) == 1 and whole.shape == (6, 2)
    assert torch.equal(part, whole[[1, 3, 5]])
    ax = engine.GatherAxes(np.arange(3.0), np.arange(2.0))
    own = engine._OwnAxes([ax, ax, ax])
    a1 = own[1]
    a1.gather_x_axis[0] = 7.0
    assert own[1] is a1 and own[0].gather_x_axis[0] == 0.0 and ax.gather_x_axis[0] == 0.0
    assert len(list(own)) == 3 and own[-1] is own[2] and [a is b for a, b in zip(own[0:2], own[0:2])] == [True, True]


def test_trajectory_packing_and_host_status(monkeypatch):
    """plan.pack_trajectories_checked on the host (the upload stubbed): each row is its trajectory sorted as
    interp1d's stable mergesort, zero padded, and its status is 1 exactly when fewer than 2 points remain
    strictly ascending after the sort (repeats and NaN included) -- the rule dvh_pass_geometry applies."""
    from das_diff_veh_amd import device, plan
    monkeypatch.setattr(device, "upload", lambda arrs, dev: [np.asarray(a) for a in arrs])
    rng = np.random.default_rng(0)
    trks = []
    for i in range(200):
        k = int(rng.integers(0, 25))
        x = np.sort(rng.uniform(0, 100, k))
        if i % 7 == 0:
            x = x[::-1].copy()
        if i % 11 == 0 and k > 3:
            x[2] = x[1]
        if i % 13 == 0 and k > 3:
            x[3] = np.nan
        if i % 17 == 0:
            x = rng.permutation(x)
        trks.append((x, rng.uniform(0, 5, k)))
    for group in (trks, [t for t in trks if len(t[0]) == 9] or trks[:1]):  # mixed lengths; one length
        (tx, tt, ln), bad = plan.pack_trajectories_checked(group, "cpu")
        for i, (vx, vt) in enumerate(group):
            k = len(vx)
            o = np.argsort(vx, kind="stable")
            sx = vx[o]
            assert np.array_equal(tx[i, :k], sx, equal_nan=True) and np.array_equal(tt[i, :k], vt[o])
            assert not np.any(tx[i, k:]) and ln[i] == k
            assert bad[i] == int(k < 2 or not np.all(sx[1:] > sx[:-1]))


def test_abandoned_staging_is_drained(monkeypatch):
    """engine._stacked (host logic, staging stubbed): an error raised after the window copies started -- here the
    gather-shape check -- waits for every staging before it propagates (no copy may keep writing
    memory the caller has released, nor the shared pinned buffers the next staging uses)."""
    from das_diff_veh_amd import engine
    from das_diff_veh_amd.plan import VsgParams

    class FakeStaging:
        def __init__(self):
            self.drained = False

        def __call__(self):
            raise AssertionError("the batch must not be used after the error")

        def drain(self):
            self.drained = True
    made = []

    def fake_stage(windows, idx, device):
        made.append(FakeStaging())
        return made[-1]
    monkeypatch.setattr(engine, "_stage", fake_stage)
    wins, _ = _failing_windows()
    wins = [wins[0], wins[4]]
    prm = VsgParams(pivot=700, start_x=500, end_x=900, include_other_side=True, norm=False)
    monkeypatch.setattr(engine, "_groups", lambda w, p: ({(1,) + (10, 500, 250): [0], (1,) + (11, 500, 250): [1]},
                                                        [None, None]))
    with pytest.raises(ValueError, match="broadcast"):
        engine._stacked(wins, prm, None, 1, "cpu", 8, None)
    assert len(made) == 1 and made[0].drained
    # groups of different data shapes: one staging per group, every one drained
    made.clear()
    wins2 = [wins[0], engine.GatherAxes(None, None)]
    wins2[1].data = np.zeros((3, 4), np.float32)
    monkeypatch.setattr(engine, "_plan", lambda *a: (_ for _ in ()).throw(ValueError("bad trajectory")))
    monkeypatch.setattr(engine, "_groups", lambda w, p: ({((60, 5500), 10, 500, 250): [0], ((3, 4), 10, 500, 250): [1]},
                                                        [None, None]))
    with pytest.raises(ValueError, match="bad trajectory"):
        engine._stacked(wins2, prm, None, 1, "cpu", 8, None)
    assert len(made) == 2 and all(m.drained for m in made)


def test_switch_interval_is_opt_in_and_refcounted(monkeypatch):
    """engine.stacked leaves the interpreter's switch interval alone unless DVH_SWITCH_INTERVAL asks; when asked,
    overlapping calls restore the caller's interval only when the last one ends."""
    import sys
    import threading

    from das_diff_veh_amd import engine
    prev = sys.getswitchinterval()
    monkeypatch.setattr(engine, "_SWITCH", 0.0)
    with engine._switch_interval():
        assert sys.getswitchinterval() == prev
    monkeypatch.setattr(engine, "_SWITCH", 1e-4)
    inside, go = threading.Event(), threading.Event()

    def other():
        with engine._switch_interval():
            inside.set()
            go.wait(5)
    th = threading.Thread(target=other)
    with engine._switch_interval():
        assert sys.getswitchinterval() == pytest.approx(min(prev, 1e-4))
        th.start()
        inside.wait(5)
    assert sys.getswitchinterval() == pytest.approx(min(prev, 1e-4))  # the other call is still inside
    go.set()
    th.join()
    assert sys.getswitchinterval() == prev


def test_sos_pole_radius_matches_numpy_roots():
    """dvh_sos_pole_radius (host arithmetic, no GPU): the largest |pole| of a design's sections, the quantity that
    picks sosfiltfilt's matrix-pipe form (include/dvh.h DVH_SOS_MFMA_MAX_POLE)."""
    from das_diff_veh_amd import _lib
    from das_diff_veh_amd.preprocess import butter_bandpass_sos
    for dt, flo, fhi in ((0.004, 1.2, 30), (0.004, 0.08, 1), (0.002, 1, 30), (0.004, 5, 60)):
        sos = np.ascontiguousarray(butter_bandpass_sos(dt, flo, fhi), dtype=np.float64)
        ref = max(np.abs(np.roots(s[3:])).max() for s in sos)
        got = _lib.load().dvh_sos_pole_radius(sos.ctypes.data, len(sos))
        assert abs(got - ref) < 1e-12, (dt, flo, fhi, got, ref)
    assert _lib.load().dvh_sos_pole_radius(None, 3) == -1.0


def test_sosfiltfilt_rejects_misaligned_workspace():
    """The state scans move 16-byte pieces of the workspace: a misaligned one is an argument error, reported before
    any device work (no GPU needed to check it)."""
    from das_diff_veh_amd import _lib
    lib = _lib.load()
    fake = ctypes.c_void_p(0x1000)
    for name, extra in (("dvh_sosfiltfilt", ()), ("dvh_sosfiltfilt_planned", (None,))):
        args = (fake, 0, 4, 3000, 3000, fake, 10, 63, fake) + extra + (ctypes.c_void_p(0x1008), None)
        assert getattr(lib, name)(*args) == -2
        assert b"16-byte aligned" in lib.dvh_last_error()


def test_save_images_raises_before_imaging():
    """save_images (apis/imaging_classes.py:110-117) points at the reference's plotting with no device work, also on
    the sharded flavour-B path whose per-pass images are never formed (images is None)."""
    from das_diff_veh_amd.apis.imaging_classes import DispersionImagesFromWindows, VirtualShotGathersFromWindows
    d = DispersionImagesFromWindows([])
    d.images = None
    with pytest.raises(NotImplementedError, match="were not formed"):
        d.save_images("/nonexistent")
    with pytest.raises(NotImplementedError, match="plot_xcorr"):
        VirtualShotGathersFromWindows([]).save_images("/nonexistent")


def test_workflow_requires_imaging_kwargs():
    """ImagingWorkflowOneDirectory.imaging (apis/imaging_workflow.py:33-80) with the reference's default
    imaging_kwargs=None fails as the reference's get_images(**None) does, before any record is read."""
    from das_diff_veh_amd.apis.imaging_workflow import ImagingWorkflowOneDirectory
    wf = ImagingWorkflowOneDirectory(iter(()), [], method="xcorr")
    with pytest.raises(TypeError):
        wf.imaging(595, 700, 620)
    with pytest.raises(NotImplementedError):
        wf.plot_avg_images()
