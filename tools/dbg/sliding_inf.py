"""Debug: which sliding units disagree with the oracle on the inf / NaN pattern, and why."""
import sys
import numpy as np
sys.path.insert(0, ".")
import torch
from tests.test_sliding_gpu import _case, _oracle_unit
from das_diff_veh_amd import vsg
from das_diff_veh_amd.plan import UnitPlan, VsgParams

dev = torch.device("cuda", 0)
kw = dict(include_other_side=True, norm=False)
w, x, t, trk = _case(dev, n=3)
pch = np.arange(32, w.shape[1] - 32, 8)
plan = UnitPlan.sliding(x, t, trk, pch, 200.0, VsgParams(**kw), full_only=False)
flat = vsg.flat_units(w, plan)
sc = vsg.vsg_scales(flat, plan, win_sumsq=vsg.unit_sumsq(vsg.window_sumsq(w), plan))
got = vsg.vsg_gathers(flat, plan, sc).double().cpu().numpy()
scn = sc.cpu().numpy()
host = w.double().cpu().numpy()
bad = 0
for u in range(plan.n_pass):
    with np.errstate(all="ignore"):
        ref = _oracle_unit(host, x, t, trk, plan, u, kw)
    same = all(np.array_equal(fn(got[u]), fn(ref)) for fn in (np.isnan, np.isposinf, np.isneginf))
    if not same:
        bad += 1
        if bad <= 4:
            piv_row = plan.pass_tab[u, 1] - plan.pass_tab[u, 0]
            print("unit", u, "win", plan.unit_window[u], "pivot", plan.unit_pivot[u], "piv_row", piv_row, "scales", scn[u])
            print("  seg pivot row", plan.seg_tab[u, piv_row].tolist())
            for r in range(plan.R):
                gi, ri = np.isinf(got[u][r]).sum(), np.isinf(ref[r]).sum()
                gn, rn = np.isnan(got[u][r]).sum(), np.isnan(ref[r]).sum()
                if (gi, gn) != (ri, rn):
                    print("  row", r, "seg", plan.seg_tab[u, r].tolist(), "got inf/nan", gi, gn, "ref", ri, rn,
                          "got", got[u][r][:3], "ref", ref[r][:3])
print("bad units", bad, "of", plan.n_pass)
