import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from tests import golden_io as gio
from das_diff_veh_amd import engine
from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
from das_diff_veh_amd.plan import VsgParams
from oracle import vsg as ovsg
KW = dict(pivot=700, start_x=500, end_x=900, wlen=2)
g = gio.load("vsg_w500"); n = gio.n_pass(g)
wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(n)]
slots = np.array([i % 2 for i in range(n)])
for kw in [dict(include_other_side=False), dict(include_other_side=False, norm=False)]:
    prm = VsgParams(**kw, **KW)
    for paired in ("1", "0"):
        os.environ["DVH_PAIRED"] = paired
        got, _ = engine.stacked(wins, prm, slots=slots, n_slot=2, device=torch.device("cuda:0"), chunk=2)
        got = got.double().cpu().numpy()
        for s in range(2):
            refs = []
            for i in np.where(slots == s)[0]:
                with np.errstate(all="ignore"):
                    refs.append(ovsg.virtual_shot_gather(gio.oracle_window(g, i), **kw, **KW)[0])
            with np.errstate(all="ignore"):
                ref = ovsg.stack(refs)
            gn = np.where(np.isnan(got[s]).any(1))[0].tolist(); rn = np.where(np.isnan(ref).any(1))[0].tolist()
            gp = np.where(np.isnan(got[s]).all(1))[0].tolist()
            m = np.isfinite(ref) & np.isfinite(got[s])
            err = np.abs(got[s][m] - ref[m]).max() / np.abs(ref[m]).max()
            print(kw, "paired", paired, "slot", s, "got nan rows", gn, "all-nan", gp, "ref nan rows", rn, "err", err)
