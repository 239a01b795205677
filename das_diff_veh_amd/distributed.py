"""Multi-GPU data parallelism over vehicle passes (one process per GPU, torch.distributed / RCCL).

Passes are independent units (the reference's loop apis/imaging_classes.py:99-104 is
embarrassingly parallel), so each rank images its own shard of passes, every pass weighted by
1 / GLOBAL class count, and ONE all-reduce (SUM) over xGMI turns the partial sums into the class
means (``sharded_class_means``).  Both imaging flavours use it:
  * VSG (flavour A): partial class stacks [n_class, R, w] from the fused correlate-and-stack kernel;
    the dispersion images are then computed from the reduced stacks on every rank (replicated).
  * per-pass f-v (flavour B, DispersionImagesFromWindows / TimeLapseImaging 'surface_wave',
    apis/imaging_classes.py:120-126): the f-v sampling after |FK| is linear, so each rank sums its
    passes' weighted |FK| grids per class [n_class, n_k, n_f] (float64, the compact grid the f-v
    queries touch) and the reduced grids are sampled once.
There is no other exchange on the data path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_passes(slots, world, rank):
    """Indices of the passes owned by `rank`: the passes sorted by class are dealt round-robin, so every
    rank gets the same share of every class (within one pass) and the rank totals differ by at most one
    pass (a per-class deal that always starts at rank 0 would give rank 0 one extra pass per class)."""
    slots = np.asarray(slots)
    order = np.argsort(slots, kind="stable")
    return np.sort(order[rank::world])


def global_counts(slots, n_slot):
    return np.bincount(np.asarray(slots, dtype=np.int64), minlength=n_slot)


def world_rank(group=None):
    """(world size, rank) of the group, (1, 0) without an initialised process group."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def allreduce_stacks(stacks, group=None):
    """In-place SUM of a list of same-dtype tensors across ranks with one bucketed collective.
    Device tensors under a gloo group (e.g. several ranks sharing one GPU) are reduced through host
    copies; under RCCL they are reduced where they are."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return stacks
    if dist.get_backend(group) == "gloo" and any(t.is_cuda for t in stacks):
        host = [t.detach().cpu() for t in stacks]
        allreduce_stacks(host, group)
        for t, h in zip(stacks, host):
            t.copy_(h)
        return stacks
    if len(stacks) == 1 and stacks[0].is_contiguous():  # one resident buffer: reduce in place
        dist.all_reduce(stacks[0], op=dist.ReduceOp.SUM, group=group)
        return stacks
    flat = torch.cat([t.reshape(-1) for t in stacks])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for t in stacks:
        n = t.numel()
        t.view(-1).copy_(flat[off:off + n])
        off += n
    return stacks


def sharded_class_means(partial, slots, n_slot, group=None):
    """The one-exchange pattern of the sharded imaging job.  ``slots`` [n]: the class of every pass of
    the WHOLE job (every rank holds the same list).  This rank takes its share (shard_passes) and calls
    ``partial(mine, weights)``, which must return a tensor whose leading axis is the class slot holding
    sum_{p in mine} weights[p] * image_p per class, with weights = 1 / global class count.  One
    all_reduce(SUM) of that tensor gives every rank the class means sum(images) / len(images)
    (apis/imaging_classes.py:106-107).  Returns (means, mine)."""
    slots = np.asarray(slots, dtype=np.int64)
    if slots.size and (slots.min() < 0 or slots.max() >= n_slot):
        raise ValueError("class slot out of range [0, n_slot)")  # same list on every rank: all raise
    world, rank = world_rank(group)
    counts = global_counts(slots, n_slot)
    mine = shard_passes(slots, world, rank).astype(np.int64)
    weights = 1.0 / counts[slots[mine]] if mine.size else np.zeros(0)
    # a pass only its owner images can fail (a trajectory interp1d rejects, a mute table, ...): every rank
    # learns of it before the data all-reduce, so no rank is left waiting in the collective
    err = None
    try:
        part = partial(mine, weights)
        if part.shape[0] != n_slot:
            raise ValueError("partial() must return per-slot sums [n_slot, ...]")
    except Exception as e:  # noqa: BLE001 -- re-raised below, on this rank and (as a RuntimeError) on the others
        err = e
    failed = any_rank_failed(err is not None, group)
    if err is not None:
        raise err
    if failed:
        raise RuntimeError(f"sharded imaging failed on another rank (rank {failed - 1}); see its error")
    allreduce_stacks([part], group)
    return part, mine


def any_rank_failed(mine_failed, group=None):
    """0 when no rank of the group failed, else 1 + the lowest failing rank (one small all-reduce)."""
    world, rank = world_rank(group)
    if world == 1:
        return 1 if mine_failed else 0
    dev = None
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    code = (world - rank) if mine_failed else 0  # MAX picks the lowest failing rank
    t = torch.tensor([code], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    v = int(t.item())
    return 0 if v == 0 else world - v + 1


def max_over_ranks(value, device=None, group=None):
    if not dist.is_available() or not dist.is_initialized():
        return value
    if dist.get_backend(group) == "gloo":
        device = None  # gloo reduces host tensors
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
