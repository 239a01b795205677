"""World-size-2 gloo test (CPU) of the flavour-B exchange: each rank forms its shard's weighted per-pass
f-v sums (the oracle stands in for the kernels here: naive dispersion of the trajectory-muted windows,
apis/imaging_classes.py:120-126), distributed.sharded_class_means all-reduces them, and every rank must
hold the reference's DispersionImagesFromWindows mean (tests/golden/disp.npz:muted_stack).  On the GPU
box the same exchange runs on |FK| grids from the HIP kernels (tests/test_distributed_gpu.py)."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import golden_io as gio


def _fv(i):
    from oracle import disp, preprocess
    g = gio.load("disp")
    w = gio.oracle_window(g, i)
    m = preprocess.mute_along_traj(w["data"], w["x_axis"], w["t_axis"], w["veh_state_x"], w["veh_state_t"], 300)
    return disp.naive_disp(m, w["x_axis"], w["t_axis"], g["freqs"], g["vels"], 500, 800, norm=False)


def _worker(rank, world, port, slots, n_slot, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from das_diff_veh_amd.distributed import sharded_class_means

        def partial(mine, weights):
            out = torch.zeros((n_slot, 500, 242), dtype=torch.float64)
            for i, wt in zip(mine, weights):
                out[slots[i]] += torch.from_numpy(_fv(int(i)).astype(np.float64)) * wt
            return out

        means, mine = sharded_class_means(partial, slots, n_slot)
        q.put((rank, means.numpy(), mine.tolist()))
    finally:
        dist.destroy_process_group()


def _run(world, slots, n_slot):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, slots, n_slot, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=300) for _ in range(world)), key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_two_rank_flavour_b_means_equal_reference():
    g = gio.load("disp")
    out = _run(2, np.zeros(3, dtype=np.int64), 1)
    assert sorted(out[0][2] + out[1][2]) == [0, 1, 2]
    for _, means, _ in out:
        ref = g["muted_stack"].astype(np.float64)
        assert np.abs(means[0] - ref).max() <= 1e-6 * np.abs(ref).max()


def test_three_ranks_two_classes_one_rank_empty_class():
    """3 passes, classes {0, 1, 0} over 3 ranks: a rank may hold no pass of a class (or none at all) and
    still joins the one collective; class means use the global counts."""
    slots = np.array([0, 1, 0])
    out = _run(3, slots, 2)
    fv = [_fv(i).astype(np.float64) for i in range(3)]
    for _, means, _ in out:
        assert np.abs(means[0] - (fv[0] + fv[2]) / 2).max() <= 1e-9 * np.abs(fv[0]).max()
        assert np.abs(means[1] - fv[1]).max() <= 1e-9 * np.abs(fv[1]).max()
