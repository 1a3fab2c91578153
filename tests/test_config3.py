"""Config 3 (BASELINE.json configs[2]): Zipf message sizes 64 B - 1 MiB split
into TEXT/BINARY + CONTINUATION fragments (optionally with interleaved PINGs),
serialized bit-exact vs the reference (SHA-256 of the reference's own wire
output, tests/golden/zipf_digests.json) and reassembled on deserialize.

CPU tests pin the oracle and the schedule generator; GPU tests run the
device codec at 64 MiB and at the full 4 GiB."""
import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import golden, gpu_present
from coldforce_amd import workloads as W


def sha(b) -> str:
    return hashlib.sha256(b.tobytes() if hasattr(b, "tobytes") else b).hexdigest()


def build(g):
    desc, msgs = W.zipf_batch(g["target_bytes"], g["seed"], g["key_seed"], ping_every=g["ping_every"])
    assert len(desc) == g["n_frames"] and len(msgs["len"]) == g["n_messages"]
    assert [int(x) for x in msgs["len"][:16]] == g["first_message_sizes"]
    assert msgs["arena_bytes"] == g["arena_bytes"]
    return desc, msgs


def arena_np(g):
    n = g["arena_bytes"]
    return O.splitmix_words(g["seed"], 0, (n + 7) // 8).view(np.uint8)[:n]


@pytest.mark.parametrize("idx", [0, 1])
def test_oracle_zipf_digest_and_reassembly(idx):
    g = golden("zipf_digests.json")[idx]
    desc, msgs = build(g)
    arena = arena_np(g)
    assert sha(arena) == g["arena_sha256"]
    d = desc.copy()
    d["mask_key"] = O.keys(g["key_seed"], len(d))       # the reference's key stream
    assert np.array_equal(d["mask_key"], desc["mask_key"])
    wire, d2 = O.serialize_batch(arena, d.view(O.DESC_DTYPE))
    assert len(wire) == g["wire_len"] and sha(wire) == g["wire_sha256"]
    out, dd, st, total = O.deserialize_batch(wire, d2["wire_off"], capacity=len(arena) + 64,
                                             flags=O.DESERIALIZE_REASSEMBLE)
    assert (st == 0).all() and total == len(arena)
    data = msgs["data_bytes"]
    # data frames packed in stream order == the messages back to back
    assert np.array_equal(out[:data], arena[:data])
    # control frames after all data bytes, in stream order
    ctl = (d["opcode"] & 8) != 0
    assert ctl.sum() == msgs["pings"]
    assert np.array_equal(out[data:total], arena[data:])
    for m in range(0, len(msgs["len"]), 97):
        f = msgs["first_frame"][m]
        assert int(dd["payload_off"][f]) == int(msgs["off"][m])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("idx", [0, 1, 2])
def test_gpu_zipf_serialize_reassemble(idx):
    import torch
    from coldforce_amd import cfws
    cfws.init()
    g = golden("zipf_digests.json")[idx]
    desc, msgs = build(g)
    n_arena = g["arena_bytes"]
    payload = torch.empty(W.round16(n_arena) + 16, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(payload, g["seed"])
    d_t = cfws.desc_to_device(desc)
    offs, total = W.wire_layout(desc)
    assert total == g["wire_len"]
    wire = torch.empty(W.round16(total), dtype=torch.uint8, device="cuda")
    tot = cfws.serialize(payload, d_t, wire)
    torch.cuda.synchronize()
    assert tot.item() == total
    h = hashlib.sha256()
    for o in range(0, total, 1 << 28):
        h.update(wire[o:min(total, o + (1 << 28))].cpu().numpy().tobytes())
    assert h.hexdigest() == g["wire_sha256"]
    idx_t = torch.from_numpy(offs.astype(np.int64)).cuda()
    out = torch.empty(W.round16(n_arena) + 64, dtype=torch.uint8, device="cuda")
    d2, st, ptot = cfws.deserialize(wire, total, idx_t, out, flags=cfws.DESERIALIZE_REASSEMBLE)
    torch.cuda.synchronize()
    assert ptot.item() == n_arena and bool((st == 0).all())
    assert torch.equal(out[:n_arena], payload[:n_arena])
    if idx < 2:   # the per-frame descriptors against the oracle too
        e_out, e_d, e_st, e_tot = O.deserialize_batch(
            np.frombuffer(wire[:total].cpu().numpy().tobytes(), np.uint8), offs,
            capacity=out.numel(), flags=O.DESERIALIZE_REASSEMBLE)
        got = cfws.desc_from_device(d2)
        for f in ("payload_off", "payload_size", "fin", "opcode", "mask_key", "header_size"):
            assert np.array_equal(got[f], e_d[f]), f
