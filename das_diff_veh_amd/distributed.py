"""Multi-GPU data parallelism over vehicle passes (one process per GPU, torch.distributed / RCCL).

Passes are independent units (the reference's loop apis/imaging_classes.py:99-104 is
embarrassingly parallel), so each rank images its own shard of passes with the fused
correlate-and-stack kernel, every pass weighted by 1 / GLOBAL class count, and ONE all-reduce
(SUM) of the flat partial class stacks over xGMI turns the partial sums into the class means.
The dispersion images are then computed from the reduced stacks on every rank (replicated; they
are a few tens of microseconds of work).  There is no other exchange on the data path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_passes(slots, world, rank):
    """Indices of the passes owned by `rank`: each class dealt round-robin, so every rank gets the
    same share of every class (load balance and identical per-class work)."""
    slots = np.asarray(slots)
    idx = []
    for s in np.unique(slots):
        members = np.flatnonzero(slots == s)
        idx.append(members[rank::world])
    return np.sort(np.concatenate(idx)) if idx else np.zeros(0, dtype=np.int64)


def global_counts(slots, n_slot):
    return np.bincount(np.asarray(slots, dtype=np.int64), minlength=n_slot)


def allreduce_stacks(stacks, group=None):
    """In-place SUM of a list of same-dtype tensors across ranks with one bucketed collective."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
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


def max_over_ranks(value, device=None, group=None):
    if not dist.is_available() or not dist.is_initialized():
        return value
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
