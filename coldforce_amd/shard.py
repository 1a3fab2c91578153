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


def byte_shard_range(msg_off: np.ndarray, total_bytes: int, rank: int,
                     world_size: int) -> tuple[int, int]:
    """Contiguous messages [m0, m1) for `rank` when a batch of messages (their
    payload offsets msg_off, back to back, total_bytes in all) is split by
    cumulative payload bytes: rank g owns the
    messages that start in [g*T/G, (g+1)*T/G). Cuts fall on message
    boundaries, so every continuation sequence stays on one GPU."""
    lo = total_bytes * rank // world_size
    hi = total_bytes * (rank + 1) // world_size
    m0 = int(np.searchsorted(msg_off, np.uint64(lo), side="left"))
    m1 = int(np.searchsorted(msg_off, np.uint64(hi), side="left"))
    return m0, m1


def zipf_shard(bytes_per_rank: int, rank: int, world_size: int, seed: int, key_seed: int):
    """The rank's byte-balanced share of one global config-3 batch of
    bytes_per_rank x world_size payload bytes. Keys are the global random()
    stream's slice, payload bytes the global arena's, so the union of the
    shards is the single-process batch (and world_size 1 is config 3
    itself). Returns (desc with rank-local payload_off, messages with
    rank-local offsets and frame numbers, payload byte_base of the shard)."""
    desc, msgs = W.zipf_batch(bytes_per_rank * world_size, seed, key_seed)
    m0, m1 = byte_shard_range(msgs["off"], msgs["data_bytes"], rank, world_size)
    n_msg = len(msgs["off"])
    f0 = int(msgs["first_frame"][m0]) if m0 < n_msg else len(desc)
    f1 = int(msgs["first_frame"][m1]) if m1 < n_msg else len(desc)
    base = int(msgs["off"][m0]) if m0 < n_msg else msgs["data_bytes"]
    end = int(msgs["off"][m1]) if m1 < n_msg else msgs["data_bytes"]
    d = desc[f0:f1].copy()
    d["payload_off"] -= np.uint64(base)
    local = dict(off=msgs["off"][m0:m1] - np.uint64(base), len=msgs["len"][m0:m1],
                 opcode=msgs["opcode"][m0:m1], first_frame=msgs["first_frame"][m0:m1] - f0,
                 n_frames=msgs["n_frames"][m0:m1], arena_bytes=end - base,
                 data_bytes=end - base, pings=0)
    return d, local, base


def _coll_device(device):
    """Where a bookkeeping collective's tensor lives: the rank's GPU under
    RCCL, the host under gloo (a multi-rank rehearsal on fewer GPUs)."""
    import torch.distributed as dist
    return "cpu" if dist.get_backend() == "gloo" else device


def gather_floats(values, device=None) -> list[list[float]]:
    """Every rank's `values` (a few floats: timings, byte counts), rank order.
    Bookkeeping only; the data path has no collective."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [list(map(float, values))]
    t = torch.tensor(list(values), dtype=torch.float64, device=_coll_device(device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.tolist()] for o in out]


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


__all__ = ["world", "shard_range", "uniform_shard", "byte_shard_range", "zipf_shard", "gather_floats",
           "max_over_ranks", "sum_over_ranks", "W"]
