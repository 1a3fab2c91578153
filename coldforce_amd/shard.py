"""Frame-batch sharding across GPUs: one process per GPU,
each rank owns a contiguous range of a global frame batch, no data-path
collective. Ranks only meet for a barrier and a max-over-ranks of their
elapsed time (bench timing), which works over gloo (CPU tests) and RCCL.
"""
from __future__ import annotations

import os

import numpy as np

from . import cfws
from . import workloads as W


def world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def shard_range(n_total: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous [first, first + count) of n_total frames for `rank`."""
    base, rem = divmod(n_total, world_size)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def uniform_shard(frames_per_rank: int, frame_size: int, key_seed: int, rank: int,
                  world_size: int):
    """The rank's slice of a global uniform batch of frames_per_rank x
    world_size frames. Keys are the global random() stream's slice, so the
    union of all shards is exactly the single-process batch. Returns
    (desc with rank-local payload_off, payload byte_base of the shard)."""
    n_total = frames_per_rank * world_size
    first, count = shard_range(n_total, rank, world_size)
    keys = cfws.draw_mask_keys(n_total, seed=key_seed)[first:first + count]
    d = np.zeros(count, dtype=cfws.DESC_DTYPE)
    d["payload_off"] = np.arange(count, dtype=np.uint64) * np.uint64(frame_size)
    d["payload_size"] = frame_size
    d["fin"], d["opcode"], d["mask"] = 1, cfws.OPCODE_BINARY, 1
    d["mask_key"] = keys
    return d, first * frame_size


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


__all__ = ["world", "shard_range", "uniform_shard", "max_over_ranks", "sum_over_ranks", "W"]
