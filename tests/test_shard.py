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


@pytest.mark.parametrize("world", [2, 8])
def test_shards_union_equals_single_batch(world):
    """world 8 rehearses the driver's 8-GPU launch shape on CPU (gloo)."""
    import torch.multiprocessing as mp
    F, fs = 48, 1000
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
    assert tmax == float(world) and ok


def test_byte_shard_range_balanced():
    """Config 3's split: contiguous messages, cuts on message
    boundaries, byte shares within one message (<= 1 MiB) of T/G."""
    from coldforce_amd import workloads as W
    _, msgs = W.zipf_batch(64 << 20, 0x5EED0003, 3)
    T, n = msgs["data_bytes"], len(msgs["off"])
    for w in (1, 2, 3, 8):
        at = 0
        for r in range(w):
            m0, m1 = shard.byte_shard_range(msgs["off"], T, r, w)
            assert m0 == at
            at = m1
            got = int(msgs["len"][m0:m1].sum())
            assert abs(got - T / w) <= 1 << 20, (w, r, got)
        assert at == n


def _zipf_rank_main(rank, world, port, per_rank, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    desc, msgs, base = shard.zipf_shard(per_rank, rank, world, 0x5EED0003, 3)
    arena = O.fill_splitmix(msgs["arena_bytes"], 0x5EED0003, base)
    wire, d2 = O.serialize_batch(arena, desc.view(O.DESC_DTYPE))
    # each shard reassembles on its own: its messages back to back
    out, _, st, total = O.deserialize_batch(wire, d2["wire_off"], capacity=len(arena) + 64,
                                            flags=O.DESERIALIZE_REASSEMBLE)
    ok = bool((st == 0).all()) and total == len(arena) and np.array_equal(out[:total], arena)
    parts = [None] * world
    dist.all_gather_object(parts, wire.tobytes())
    rows = shard.gather_floats([rank, len(desc), msgs["data_bytes"]])
    if rank == 0:
        q.put((b"".join(parts), rows, ok))
    dist.destroy_process_group()


def test_zipf_shards_union_equals_single_batch():
    """World size 2 over gloo: each rank's byte-balanced share of the global
    config-3 batch; the shards' wires joined equal the single-process wire,
    and gather_floats returns every rank's row in rank order."""
    import torch.multiprocessing as mp
    from coldforce_amd import workloads as W
    per_rank, world = 8 << 20, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zipf_rank_main, args=(r, world, port, per_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    joined, rows, ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    desc, msgs = W.zipf_batch(per_rank * world, 0x5EED0003, 3)
    wire, _ = O.serialize_batch(O.fill_splitmix(msgs["arena_bytes"], 0x5EED0003, 0),
                                desc.view(O.DESC_DTYPE))
    assert hashlib.sha256(joined).hexdigest() == hashlib.sha256(wire.tobytes()).hexdigest()
    assert ok
    assert [r[0] for r in rows] == [0.0, 1.0]
    assert sum(r[1] for r in rows) == len(desc)
    assert sum(r[2] for r in rows) == msgs["data_bytes"]


def test_bench_per_gpu_rows():
    """bench.py's per-GPU rows: each rank's payload rate over its own span and
    its slower execute against the HBM peak."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rows = bench.per_gpu_rows([[0.5, 1 << 30, 1.0, 2.0, 8e9], [1.0, 1 << 30, 1.0, 1.0, 8e9]], 10)
    assert [r["rank"] for r in rows] == [0, 1]
    assert rows[0]["GiBps"] == 40.0 and rows[1]["GiBps"] == 20.0
    assert rows[0]["execute_GBps"] == 4000.0 and rows[0]["frac"] == 0.5
    assert rows[1]["frac"] == 1.0
    assert "frac" not in bench.per_gpu_rows([[1.0, 1 << 30]], 1)[0]
