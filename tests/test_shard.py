"""Multi-GPU path on CPU: one process per rank over gloo (world size 2), each
rank owning a contiguous shard of one global frame batch. The union of the
shards must be byte-identical to the single-process batch (the reference's
sequential serialize of all frames), and the timing reduction must be a max."""
import hashlib
import os
import socket

import numpy as np
import pytest

import oracle as O
from coldforce_amd import shard

torch = pytest.importorskip("torch")


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 65536, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, w) for r in range(w)]
            at = 0
            for first, count in spans:
                assert first == at
                at += count
            assert at == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, F, fs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    desc, byte_base = shard.uniform_shard(F, fs, 3, rank, world)
    payload = O.fill_splitmix(len(desc) * fs, 0x5EED, byte_base)
    wire, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    parts = [None] * world
    dist.all_gather_object(parts, wire.tobytes())
    t = shard.max_over_ranks(float(rank + 1))
    ok = shard.sum_over_ranks(1.0) == world
    if rank == 0:
        q.put((b"".join(parts), t, ok))
    dist.destroy_process_group()


def test_shards_union_equals_single_batch():
    import torch.multiprocessing as mp
    F, fs, world = 48, 1000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, F, fs, q)) for r in range(world)]
    for p in procs:
        p.start()
    joined, tmax, ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: the whole batch, keys from one srandom(3) stream
    n = F * world
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * fs
    d["payload_size"], d["fin"], d["opcode"], d["mask"] = fs, 1, 2, 1
    d["mask_key"] = O.keys(3, n)
    wire, _ = O.serialize_batch(O.fill_splitmix(n * fs, 0x5EED, 0), d)
    assert hashlib.sha256(joined).hexdigest() == hashlib.sha256(wire.tobytes()).hexdigest()
    assert tmax == 2.0 and ok
