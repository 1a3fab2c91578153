"""The CPU restatement (oracle/) pinned against the reference's behaviour.

Pins: RFC 6455 section 5.7 known answers, golden vectors produced by the
reference codec itself (tests/golden/make_golden.py), and -- when
oracle/_ref is built in this container -- a live randomized comparison with
the reference compiled from /root/reference.
"""
import hashlib
import random

import numpy as np
import pytest

import oracle as O
from conftest import golden


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_rfc6455_section_5_7(oracle_lib):
    # Literal RFC 6455 examples (not from the fixture): "Hello" both ways.
    L = oracle_lib
    for hx, op, fin in (("810548656c6c6f", 1, True), ("818537fa213d7f9f4d5158", 1, True),
                        ("890548656c6c6f", 9, True), ("8a8537fa213d7f9f4d5158", 10, True)):
        r = O.ref_deserialize(L, bytes.fromhex(hx))
        assert r["rc"] == 0 and r["payload"] == b"Hello\0"
        assert r["opcode"] == op and r["fin"] == fin and r["index"] == len(hx) // 2
    a = O.ref_deserialize(L, bytes.fromhex("010348656c"))
    b = O.ref_deserialize(L, bytes.fromhex("80026c6f"))
    assert (a["fin"], a["opcode"], a["payload"]) == (False, 1, b"Hel\0")
    assert (b["fin"], b["opcode"], b["payload"]) == (True, 0, b"lo\0")
    # Re-encoding the masked example with its key gives the RFC bytes back.
    assert O.serialize_keyed(True, 1, True, 0x3D21FA37, b"Hello").hex() == "818537fa213d7f9f4d5158"


def test_rfc6455_golden(oracle_lib):
    for c in golden("rfc6455_kat.json"):
        if c["wire"] is not None:
            raw = bytes.fromhex(c["wire"])
        else:
            n = c["payload_size"]
            raw = bytes.fromhex(c["wire_spec"][:20]) + bytes([0xCD]) * n
        assert sha(raw) == c["wire_sha256"]
        r = O.ref_deserialize(oracle_lib, raw)
        assert (r["rc"], r["index"], r["fin"], r["opcode"], r["payload_size"]) == \
            (c["rc"], c["index"], c["fin"], c["opcode"], c["payload_size"]), c["name"]
        assert sha(r["payload"]) == c["payload_sha256"]


def test_serialize_golden(oracle_lib):
    for c in golden("serialize_cases.json"):
        data = O.fill_splitmix(c["n"], c["payload_seed"], c["payload_byte_base"]).tobytes()
        O.srandom(oracle_lib, c["seed"])
        w = O.ref_serialize(oracle_lib, c["fin"], c["opcode"], c["mask"], data)
        assert len(w) == c["wire_len"]
        assert w[:len(c["header_hex"]) // 2].hex() == c["header_hex"], c
        assert sha(w) == c["wire_sha256"], c
        if c["wire_hex"] is not None:
            assert w.hex() == c["wire_hex"]


def test_deserialize_golden(oracle_lib):
    for c in golden("deserialize_cases.json"):
        if c["wire_hex"] is not None:
            raw = bytes.fromhex(c["wire_hex"])
        elif c["wire_spec"] and c["wire_spec"].endswith("+zeros"):
            head = bytes.fromhex(c["wire_spec"][:-len("+zeros")])
            raw = head + bytes(c["wire_len"] - len(head))
        else:
            continue  # large plain frame: rebuilt below from its spec
        assert sha(raw) == c["wire_sha256"], c["name"]
        r = O.ref_deserialize(oracle_lib, raw, c["index"], c["max_payload"])
        got = (r["rc"], r["index"], r["fin"], r["opcode"], r["payload_size"], r["payload"] is None)
        exp = (c["rc"], c["index_out"], c["fin"], c["opcode"], c["payload_size"], c["payload_is_null"])
        assert got == exp, c["name"]
        if c["payload_sha256"] is not None:
            assert sha(r["payload"]) == c["payload_sha256"], c["name"]


def test_deserialize_golden_large_plain(oracle_lib):
    raw = O.serialize_keyed(True, 2, False, 0, b"\x5a" * 70000)
    cases = {c["name"]: c for c in golden("deserialize_cases.json")}
    for name, limit in (("plain 70000 B", O.DEFAULT_MAX_PAYLOAD), ("plain 70000 B, limit 69999", 69999)):
        c = cases[name]
        assert sha(raw) == c["wire_sha256"]
        r = O.ref_deserialize(oracle_lib, raw, 0, limit)
        assert (r["rc"], r["index"], r["payload_size"]) == (c["rc"], c["index_out"], c["payload_size"])


def test_keys_golden():
    for seed, ks in golden("keys.json").items():
        got = O.keys(int(seed), len(ks))
        assert [f"{int(k) & 0xff:02x}{int(k) >> 8 & 0xff:02x}{int(k) >> 16 & 0xff:02x}{int(k) >> 24:02x}"
                for k in got] == ks


@pytest.mark.parametrize("idx", [0, 1])
def test_batch_digest_golden(idx):
    g = golden("batch_digests.json")[idx]
    n, fs = g["n_frames"], g["frame_size"]
    payload = O.splitmix_words(g["payload_seed"], 0, n * fs // 8).view(np.uint8)
    assert sha(payload.tobytes()) == g["payload_sha256"]
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * fs
    d["payload_size"] = fs
    d["fin"], d["opcode"], d["mask"] = 1, 2, 1
    d["mask_key"] = O.keys(g["key_seed"], n)
    wire, d2 = O.serialize_batch(payload, d)
    assert len(wire) == g["wire_len"]
    assert sha(wire.tobytes()) == g["wire_sha256"]
    # and back: deserialize at the serialize offsets restores the payloads
    out, desc, st, total = O.deserialize_batch(wire, d2["wire_off"], align=1,
                                               capacity=n * fs)
    assert (st == 0).all() and total == n * fs
    assert sha(out[:total].tobytes()) == g["payload_sha256"]


def test_oracle_vs_reference_random(oracle_lib, ref_lib):
    rng = random.Random(11)
    for trial in range(300):
        n = rng.choice([0, 1, 2, 5, 125, 126, 127, 300, 65535, 65536, 65537, rng.randrange(200000)])
        data = rng.randbytes(n)
        fin, op, mask = rng.random() < .5, rng.randrange(256), rng.random() < .5
        O.srandom(oracle_lib, trial)
        a = O.ref_serialize(oracle_lib, fin, op, mask, data)
        O.srandom(ref_lib, trial)
        b = O.ref_serialize(ref_lib, fin, op, mask, data)
        assert a == b
        # random truncation / corruption of the header
        w = bytearray(a)
        if rng.random() < .3:
            w = w[:rng.randrange(2, len(w) + 1)]
        if rng.random() < .2:
            w[0] = rng.randrange(256)
        lim = rng.choice([O.DEFAULT_MAX_PAYLOAD, max(0, n - 1), n])
        assert O.ref_deserialize(oracle_lib, bytes(w), 0, lim) == \
            O.ref_deserialize(ref_lib, bytes(w), 0, lim)


def test_batch_deserialize_matches_per_frame(oracle_lib):
    rng = random.Random(3)
    frames, payloads = [], []
    for i in range(200):
        n = rng.choice([0, 1, 7, 125, 126, 1000, 65536, 70001])
        p = rng.randbytes(n)
        payloads.append(p)
        frames.append(O.serialize_keyed(rng.random() < .5, rng.randrange(16), rng.random() < .7,
                                        rng.getrandbits(32), p))
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8)
    starts, consumed = O.index_frames(wire, 1000)
    assert len(starts) == 200 and consumed == len(wire)
    for align in (1, 16, 64):
        out, desc, st, total = O.deserialize_batch(wire, starts, align=align)
        assert (st == 0).all()
        for i, p in enumerate(payloads):
            off = int(desc["payload_off"][i])
            assert out[off:off + len(p)].tobytes() == p
            r = O.ref_deserialize(oracle_lib, wire.tobytes(), int(starts[i]))
            assert r["payload_size"] == len(p) and (r["payload"] or b"\0")[:-1] == p
        assert all(int(desc["payload_off"][i]) % align == 0 for i in range(200))


def test_batch_deserialize_errors_and_capacity():
    good = O.serialize_keyed(True, 2, True, 0x01020304, bytes(range(200)))
    wire = np.frombuffer(good + bytes([0xF1, 0x05]) + good[:50], dtype=np.uint8)
    starts = np.array([0, len(good), len(good) + 2, len(wire) - 1, len(wire) + 5], dtype=np.uint64)
    out, desc, st, total = O.deserialize_batch(wire, starts, align=16)
    assert list(st) == [0, O.ERROR_INVALID_FRAME, O.PARSE_MORE_DATA, O.PARSE_MORE_DATA,
                        O.PARSE_MORE_DATA]
    assert total == 208
    # capacity 100: the 200-byte payload does not fit
    out, desc, st, total = O.deserialize_batch(wire, starts[:1], align=16, capacity=100)
    assert st[0] == O.ERROR_OUT_OF_MEMORY and total == 100 and not out[:100].any()


def _index_cases():
    g = golden("index_cases.json")
    blobs = {k: bytes.fromhex(v) for k, v in g["blobs"].items()}
    return [(c, blobs[c["blob"]][:c["size"]]) for c in g["cases"]]


@pytest.mark.parametrize("i", range(len(golden("index_cases.json")["cases"])))
def test_index_stream_matches_reference_receive_loop(i):
    """orc_index_stream == the reference's receive loop (co_ws_server.c:107-169
    around its own co_ws_frame_deserialize) on the committed streams."""
    c, data = _index_cases()[i]
    st, consumed, stop = O.index_stream(np.frombuffer(data, np.uint8), c["begin"], len(data),
                                        c["max_payload"])
    assert [int(x) for x in st] == c["starts"], c["name"]
    assert consumed == c["consumed"] and stop == c["stop"], c["name"]


def test_ws_accept_key_rfc6455_example():
    """RFC 6455 section 1.3: the example nonce's Sec-WebSocket-Accept."""
    assert O.ws_accept_key(b"dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_ws_accept_key_matches_reference_fixtures():
    for c in golden("handshake_cases.json"):
        assert O.ws_accept_key(bytes.fromhex(c["key_hex"])) == c["accept"], c["key_hex"]
