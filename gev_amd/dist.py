"""Multi-GPU plumbing for the decode path: one process per GPU.

Connections are independent byte streams, so the path shards by connection
(gev already shards connections over event loops: server.go:80-91,
load_balance.go:7-28; here the unit of placement is a GPU).  Payload bytes never
leave their GPU; the only collective is the sum of the decoded {frames,
payload bytes, errors} counts -- RCCL (torch "nccl" backend) over xGMI on the
node, gloo on the CPU in tests -- plus the max-over-ranks of the timed region.
"""
from __future__ import annotations

import os
from typing import Tuple


def env() -> Tuple[int, int, int]:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device=None) -> bool:
    """Initialise the process group when WORLD_SIZE > 1; returns whether it did."""
    import torch.distributed as dist
    world, _, _ = env()
    if world <= 1 or dist.is_initialized():
        return dist.is_initialized()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    dist.init_process_group(backend, **kw)
    return True


def backend() -> str:
    """RCCL ("nccl") on GPUs; GEV_DIST_BACKEND=gloo rehearses the multi-rank
    path with several ranks on one GPU (RCCL allows one rank per device)."""
    return os.environ.get("GEV_DIST_BACKEND", "nccl")


def _gloo_host(t):
    import torch.distributed as dist
    return dist.get_backend() == "gloo" and t.is_cuda


def reduce_counts(counts) -> None:
    """In-place sum over ranks of the int64 [frames, payload_bytes, errors] tensor."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        if _gloo_host(counts):
            c = counts.cpu()
            dist.all_reduce(c)
            counts.copy_(c)
        else:
            dist.all_reduce(counts)


def max_over_ranks(value: float, device) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        if _gloo_host(t):
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def finalize() -> None:
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def rank_seed(base: int, rank: int) -> int:
    """Weak scaling: every rank decodes its own connections' batch of the same shape."""
    return base + 7919 * rank
