"""Two ranks on the one GPU of the box (gloo for the exchange, since RCCL refuses two ranks on one
device): each rank stacks ITS shard of the passes with the HIP stack kernel, weighted by the global
class counts, and one all-reduce of the partial stacks must reproduce the single-process class
means (and the oracle).  The bench runs the same path with RCCL over xGMI, one rank per GPU."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
KW = dict(pivot=700, start_x=500, end_x=900, wlen=2)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from das_diff_veh_amd import vsg
        from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
        from das_diff_veh_amd.distributed import allreduce_stacks, global_counts, shard_passes
        from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry
        dev = torch.device("cuda", 0)
        g = gio.load("vsg_w500")
        n = gio.n_pass(g)
        slots = np.arange(n) % 2
        counts = global_counts(slots, 2)
        mine = shard_passes(slots, world, rank)
        wins = [SurfaceWaveWindow(**gio.pass_arrays(g, int(i))) for i in mine]
        prm = VsgParams(include_other_side=True, norm=False, **KW)
        plan = VsgPlan([pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, prm) for w in wins], prm,
                       wins[0].data.shape[0], wins[0].data.shape[1])
        data = torch.as_tensor(np.stack([w.data for w in wins]), device=dev)
        part = vsg.vsg_stack(data, plan, vsg.StackSchedule(slots[mine], 2, chunk=2, counts=counts))
        host = part.cpu()  # gloo reduces host tensors
        allreduce_stacks([host])
        q.put((rank, host.double().numpy(), mine.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_stack_reduction(device):
    import socket

    from das_diff_veh_amd import vsg
    from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
    from das_diff_veh_amd.plan import VsgParams, VsgPlan, pass_geometry
    from oracle import vsg as ovsg
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(out[0][2] + out[1][2]) == list(range(len(out[0][2]) + len(out[1][2])))
    # single process, all passes
    import torch
    g = gio.load("vsg_w500")
    n = gio.n_pass(g)
    slots = np.arange(n) % 2
    wins = [SurfaceWaveWindow(**gio.pass_arrays(g, i)) for i in range(n)]
    prm = VsgParams(include_other_side=True, norm=False, **KW)
    plan = VsgPlan([pass_geometry(w.x_axis, w.t_axis, w.veh_state_x, w.veh_state_t, prm) for w in wins], prm,
                   wins[0].data.shape[0], wins[0].data.shape[1])
    data = torch.as_tensor(np.stack([w.data for w in wins]), device=device)
    one = vsg.vsg_stack(data, plan, vsg.StackSchedule(slots, 2, chunk=2)).double().cpu().numpy()
    for rank, stacks, _ in out:
        assert np.abs(stacks - one).max() <= 1e-6 * np.abs(one).max(), rank
        for c in range(2):
            refs = [ovsg.virtual_shot_gather(gio.oracle_window(g, i), include_other_side=True, norm=False, **KW)[0]
                    for i in np.flatnonzero(slots == c)]
            assert gio.gather_rel_err(stacks[c], ovsg.stack(refs)) < 1e-4


def _api_worker(rank, world, port, q):
    """Both drop-in flavours with shard_over_ranks=True on the ranks of a gloo group (one GPU)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from das_diff_veh_amd.apis.data_classes import SurfaceWaveWindow
        from das_diff_veh_amd.apis.imaging_classes import DispersionImagesFromWindows, VirtualShotGathersFromWindows
        from tests.test_tli_gpu import _tli
        gd = gio.load("disp")
        wins = [SurfaceWaveWindow(**gio.pass_arrays(gd, i)) for i in range(gio.n_pass(gd))]
        imgs = DispersionImagesFromWindows(wins)
        imgs.get_images(mute_offset=300, freqs=gd["freqs"], vels=gd["vels"], method="naive", start_x=500, end_x=800,
                        shard_over_ranks=True)
        assert imgs.images is None and not any(w.muted_along_traj for w in wins)
        gv = gio.load("vsg_w500")
        vw = [SurfaceWaveWindow(**gio.pass_arrays(gv, i)) for i in range(gio.n_pass(gv))]
        vimgs = VirtualShotGathersFromWindows(vw)
        vimgs.get_images(include_other_side=True, shard_over_ranks=True, **KW)
        # TimeLapseImaging.get_images forwards the keyword to its DispersionImagesFromWindows
        import das_diff_veh_amd.apis.timeLapseImaging as tl
        orig = tl.TimeLapseImaging.get_images
        tl.TimeLapseImaging.get_images = lambda self, mute_offset=300, **kw: orig(self, mute_offset,
                                                                                  shard_over_ranks=True, **kw)
        try:
            obj, _, _ = _tli()
        finally:
            tl.TimeLapseImaging.get_images = orig
        q.put((rank, imgs.avg_image.disp.fv_map, imgs.shard.tolist(), vimgs.avg_image.XCF_out, vimgs.shard.tolist(),
               obj.images.avg_image.disp.fv_map))
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_sharded_flavours(device):
    """Flavour B (DispersionImagesFromWindows, TimeLapseImaging 'surface_wave') and flavour A
    (VirtualShotGathersFromWindows) sharded over 2 ranks: every rank's avg_image equals the reference's
    single-process result (disp.npz:muted_stack, tli.npz:fv_avg, vsg_w500.npz:stack)."""
    import socket

    from tests.test_disp_gpu import _check
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_api_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=180) for _ in range(2)), key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(out[0][2] + out[1][2]) == [0, 1, 2]
    assert sorted(out[0][4] + out[1][4]) == [0, 1, 2, 3, 4]
    gd, gv, gt = gio.load("disp"), gio.load("vsg_w500"), gio.load("tli")
    for _, fv, _, xcf, _, tfv in out:
        _check(fv, gd["muted_stack"])
        assert gio.gather_rel_err(xcf, gv["stack"]) < 1e-4
        _check(tfv, gt["fv_avg"])
