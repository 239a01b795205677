"""RCCL code-path check on a one-GPU box: the calls bench.py makes at N > 1 (init_process_group("nccl",
device_id=...), barrier, the in-place all-reduce of the class stacks, max over ranks, destroy), run with
as many ranks as GPUs are visible (one here).  The multi-GPU scaling run itself is the driver's.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29571 tools/rccl_smoke.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from das_diff_veh_amd.distributed import allreduce_stacks, max_over_ranks  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", device_id=device)
    world, rank = dist.get_world_size(), dist.get_rank()
    stack = torch.full((3, 1023, 500), float(rank + 1), device=device)
    dist.barrier()
    allreduce_stacks([stack])  # the bench's call (a no-op at one rank)
    dist.all_reduce(stack)      # the RCCL collective itself, on the device buffer
    stack /= world
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    ok = bool((stack == want).all())
    m = max_over_ranks(0.5 + rank, device)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print(f"rccl ok={ok} world={world} backend=nccl allreduce={float(stack[0, 0, 0])} (want {want}) max={m}")
    sys.exit(0 if ok and m == world - 0.5 else 1)


if __name__ == "__main__":
    main()
