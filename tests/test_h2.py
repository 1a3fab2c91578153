"""WebSocket over HTTP/2 (BASELINE.json configs[4]):
WS frames carried in HTTP/2 DATA frames (co_ws_http2_extension.c:134-199,
co_http2_stream.c:933-1013 and :550-608, co_http2_frame.c:33-72 and
:211-300). CPU tests pin the oracle to the reference's own DATA encoder /
decoder (tests/golden/h2_*.json); GPU tests hold the device path to both."""
import hashlib
import random

import numpy as np
import pytest

import oracle as O
from conftest import golden, gpu_present


def sha(b) -> str:
    return hashlib.sha256(b.tobytes() if hasattr(b, "tobytes") else b).hexdigest()


def wrap_desc(case):
    frames = case["frames"]
    sizes = [f["n"] for f in frames]
    arena = b"".join(O.fill_splitmix(f["n"], f["payload_seed"], f["payload_byte_base"]).tobytes()
                     for f in frames)
    d = np.zeros(len(frames), dtype=O.DESC_DTYPE)
    d["payload_off"] = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64)
    d["payload_size"] = sizes
    d["fin"] = [f["fin"] for f in frames]
    d["opcode"] = [f["opcode"] for f in frames]
    d["mask"] = 1
    d["mask_key"] = O.keys(case["key_seed"], len(frames))
    return np.frombuffer(arena, np.uint8).copy(), d


def test_oracle_wrap_golden():
    for case in golden("h2_cases.json")["wrap"]:
        arena, d = wrap_desc(case)
        h2, _ = O.h2_serialize_batch(arena, d, case["sid"], case["max_frame"])
        assert len(h2) == case["h2_len"] and sha(h2) == case["h2_sha256"]


def test_oracle_recv_golden():
    # reference rc 0 on a non-DATA frame is "not DATA" in the batch API
    for c in golden("h2_cases.json")["recv"]:
        raw = np.frombuffer(bytes.fromhex(c["raw_hex"]), np.uint8).copy()
        r = O.h2_deserialize_batch(raw, np.array([0], np.uint64))
        exp = 3 if (c["rc"] == 0 and c["type"] != 0) else c["rc"]
        assert r["h2_status"][0] == exp, c["name"]
        if exp == 0:
            assert r["pool"][:len(c["payload_hex"]) // 2].tobytes().hex() == c["payload_hex"]


def test_oracle_messages_golden():
    g = golden("h2_cases.json")["messages"][0]
    stream = np.frombuffer(bytes.fromhex(g["stream_hex"]), np.uint8).copy()
    r = O.h2_deserialize_batch(stream, O.h2_index(stream), g["max_frame"], align=1)
    assert r["n_msg"] == len(g["results"])
    for k, e in enumerate(g["results"]):
        d = r["msg_desc"][k]
        assert r["msg_status"][k] == e["rc"]
        assert (bool(d["fin"]), int(d["opcode"]), int(d["payload_size"])) == \
            (e["fin"], e["opcode"], e["payload_size"])
        if e["payload_sha256"]:
            o = int(d["payload_off"])
            assert sha(r["payload"][o:o + e["payload_size"]]) == e["payload_sha256"]


@pytest.mark.parametrize("idx", [0, 1])
def test_oracle_h2_digest(idx):
    g = golden("h2_digests.json")[idx]
    n, fs = g["n_frames"], g["frame_size"]
    arena = O.splitmix_words(g["payload_seed"], 0, (n * fs + 7) // 8).view(np.uint8)[:n * fs]
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * fs
    d["payload_size"], d["fin"], d["opcode"], d["mask"] = fs, 1, 2, 1
    d["mask_key"] = O.keys(g["key_seed"], n)
    h2, _ = O.h2_serialize_batch(arena, d, g["sid"], g["max_frame"])
    assert len(h2) == g["h2_len"] and sha(h2) == g["h2_sha256"]
    r = O.h2_deserialize_batch(h2, O.h2_index(h2), g["max_frame"], align=1,
                               payload_capacity=n * fs)
    assert r["n_msg"] == n and (r["msg_status"] == 0).all()
    assert np.array_equal(r["payload"][:n * fs], arena)


# ---- device ---------------------------------------------------------------------

def _gpu():
    import torch
    from coldforce_amd import cfws
    cfws.init()
    return torch, cfws


def gpu_h2_serialize(payload: np.ndarray, desc: np.ndarray, sid=1, S=16384):
    torch, cfws = _gpu()
    from coldforce_amd import workloads as W
    pay = torch.from_numpy(payload if payload.size else np.zeros(16, np.uint8)).cuda()
    d_t = cfws.desc_to_device(desc)
    _, wtotal = W.wire_layout(desc)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
    h2 = torch.full((cfws.h2_wrapped_bound(wire.numel(), len(desc), S),), 0xEE, dtype=torch.uint8,
                    device="cuda")
    tot = cfws.h2_serialize(pay, d_t, wire, h2, sid, S)
    torch.cuda.synchronize()
    t = int(tot.item())
    return h2[:t].cpu().numpy(), t


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("S", [16384, 1000, 100, 64, 63, 16])
def test_gpu_h2_serialize_random(S):
    rng = random.Random(S)
    payload = O.fill_splitmix(1 << 20, S, 0)
    n = 800
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 1, 125, 126, 999, 1000, 16376, 16384, 40000, 70000])
        d[i] = (rng.randrange(0, (1 << 20) - sz), 0, sz, rng.getrandbits(32), rng.random() < .6,
                rng.choice([0, 1, 2, 9]), rng.random() < .7, 0)
    exp, _ = O.h2_serialize_batch(payload, d, 5, S)
    got, t = gpu_h2_serialize(payload, d, 5, S)
    assert t == len(exp)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("n", [1, 255, 256, 257, 65536, 65537, 524288, 524289])
def test_gpu_h2_serialize_plan_grid_sizes(n):
    """The send plan around its block bounds (256 frames per block; past
    2,048 blocks a scan launch between reduce and apply), called twice on
    the same arenas."""
    rng = np.random.default_rng(n)
    payload = O.fill_splitmix(1 << 20, 77, 0)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_size"] = rng.choice([0, 1, 125, 126, 3000, 16376, 20000] if n < 65536 else [0, 1, 125, 126, 300], n)
    d["payload_off"] = rng.integers(0, (1 << 20) - 20000, n).astype(np.uint64)
    d["mask"] = (rng.random(n) < .7).astype(np.uint8)
    d["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * d["mask"]
    d["fin"], d["opcode"] = 1, 2
    exp, _ = O.h2_serialize_batch(payload, d, 3, 16384)
    for _ in range(2):
        got, t = gpu_h2_serialize(payload, d, 3, 16384)
        assert t == len(exp)
        assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_serialize_streams():
    """Sends queued on two streams without a synchronize between them, each
    checked against the oracle."""
    torch, cfws = _gpu()
    from coldforce_amd import workloads as W
    rng = np.random.default_rng(5)
    payload = O.fill_splitmix(1 << 20, 78, 0)
    pay = torch.from_numpy(payload).cuda()
    jobs = []
    for j in range(2):
        n = 20000 + 7 * j
        d = np.zeros(n, dtype=O.DESC_DTYPE)
        d["payload_size"] = rng.choice([0, 125, 126, 5000, 16376, 17000], n)
        d["payload_off"] = rng.integers(0, (1 << 20) - 17000, n).astype(np.uint64)
        d["mask"] = (rng.random(n) < .5).astype(np.uint8)
        d["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * d["mask"]
        d["fin"], d["opcode"] = 1, 2
        exp, _ = O.h2_serialize_batch(payload, d, 1 + j, 16384)
        _, wtotal = W.wire_layout(d)
        wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
        h2 = torch.empty(cfws.h2_wrapped_bound(wire.numel(), n, 16384), dtype=torch.uint8, device="cuda")
        jobs.append((torch.cuda.Stream(), cfws.desc_to_device(d), wire, h2, exp, 1 + j))
    torch.cuda.synchronize()
    tots = [[], []]
    for _ in range(6):
        for j, (st, d_t, wire, h2, exp, sid) in enumerate(jobs):
            with torch.cuda.stream(st):
                tots[j].append(cfws.h2_serialize(pay, d_t, wire, h2, sid, 16384, stream=st))
    torch.cuda.synchronize()
    for j, (st, d_t, wire, h2, exp, sid) in enumerate(jobs):
        assert all(int(t.item()) == len(exp) for t in tots[j])
        assert np.array_equal(h2[:len(exp)].cpu().numpy(), exp)


def _units(d, S):
    """Output lengths of the DATA frames the send makes (9 + slice)."""
    out = []
    for n, m in zip(d["payload_size"], d["mask"]):
        w = int(n) + O.header_size(int(n), bool(m))
        k = 1 if w <= S else -(-w // S)
        out += [9 + min(S, w - j * S) for j in range(k)]
    return out


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("S,case", [(16384, "mixed"), (16384, "last_short"), (5000, "mixed"),
                                    (16384, "cut"), (4200, "mixed")])
def test_gpu_h2_send_in_region_edges(S, case):
    """The fused send's in-region edge chunks (two_frame_region<kModeH2Ser,
    kEdges>): every DATA frame but the stream's last spans more than a 4 KiB
    region and a 32-byte margin (the plan's flag), so the two-frame regions
    assemble each boundary's chunks -- the previous body's tail, the DATA +
    WS header at any offset, the next body's head -- in registers. Random
    payload sizes (7/16/64-bit WS lengths, masked and unmasked, unaligned
    sources, WS frames split into several DATA frames), a short last frame,
    and a capacity cut inside the stream, against the oracle (pinned to the
    reference's co_http2_frame.c + co_ws_frame.c)."""
    rng = random.Random(S * 31 + len(case))
    payload = O.fill_splitmix(1 << 22, S, 0)
    d = []
    while len(d) < 1500:
        sz = rng.choice([rng.randrange(4200, 16300), rng.randrange(4200, 40000), 65535, 65536,
                         rng.randrange(66000, 200000)])
        m = rng.random() < .8
        w = sz + O.header_size(sz, m)
        k = 1 if w <= S else -(-w // S)
        if 9 + w - (k - 1) * S < 4096 + 32:
            continue
        d.append((rng.randrange(0, (1 << 22) - sz), 0, sz, rng.getrandbits(32) if m else 0,
                  rng.random() < .6, rng.choice([0, 1, 2, 9]), m, 0))
    if case == "last_short":
        d.append((77, 0, 10, 0x1234567, True, 2, True, 0))
    d = np.array(d, dtype=O.DESC_DTYPE)
    units = _units(d, S)
    assert min(units[:-1]) >= 4096 + 32          # the plan's flag is clear
    exp, _ = O.h2_serialize_batch(payload, d, 7, S)
    if case != "cut":
        got, t = gpu_h2_serialize(payload, d, 7, S)
        assert t == len(exp)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (bad.size, bad[:10])
        return
    torch, cfws = _gpu()
    from coldforce_amd import workloads as W
    pay = torch.from_numpy(payload).cuda()
    _, wtotal = W.wire_layout(d)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
    for cap in (len(exp) // 2 + 4101, len(exp) // 3 // 4096 * 4096):
        h2 = torch.full((cap + 4096,), 0xEE, dtype=torch.uint8, device="cuda")
        tot = cfws.h2_serialize(pay, cfws.desc_to_device(d), wire, h2[:cap], 7, S)
        torch.cuda.synchronize()
        assert int(tot.item()) == len(exp)
        got = h2.cpu().numpy()
        assert np.array_equal(got[:cap], exp[:cap]) and (got[cap:] == 0xEE).all(), cap


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_wrap_golden():
    for case in golden("h2_cases.json")["wrap"]:
        arena, d = wrap_desc(case)
        got, t = gpu_h2_serialize(arena, d, case["sid"], case["max_frame"])
        assert t == case["h2_len"] and sha(got) == case["h2_sha256"]


def gpu_h2_deserialize(h2: np.ndarray, index: np.ndarray, S=16384, align=16, pool_cap=None,
                       payload_cap=None, max_payload=O.DEFAULT_MAX_PAYLOAD):
    torch, cfws = _gpu()
    h = torch.from_numpy(np.concatenate([h2, np.zeros(16, np.uint8)])).cuda()
    idx = torch.from_numpy(index.astype(np.int64)).cuda()
    pool = torch.empty(max(pool_cap if pool_cap is not None else len(h2), 16), dtype=torch.uint8,
                       device="cuda")
    pay = torch.empty(max(payload_cap if payload_cap is not None else len(h2) + 16 * len(index) + 16,
                          16), dtype=torch.uint8, device="cuda")
    if pool_cap is not None:
        pool = pool[:pool_cap] if pool_cap else pool[:0]
    if payload_cap is not None:
        pay = pay[:payload_cap]
    st, md, ms, tot, m = cfws.h2_deserialize(h, len(h2), idx, pool, pay, S, max_payload, align)
    torch.cuda.synchronize()
    return dict(h2_status=st.cpu().numpy(), msg_desc=cfws.desc_from_device(md) if m else
                np.zeros(0, O.DESC_DTYPE), msg_status=ms.cpu().numpy(),
                payload=pay.cpu().numpy(), total=int(tot.item()), n_msg=m)


def check_h2_deserialize(h2, index, **kw):
    got = gpu_h2_deserialize(h2, index, **kw)
    exp = O.h2_deserialize_batch(h2, index, kw.get("S", 16384), kw.get("max_payload", O.DEFAULT_MAX_PAYLOAD),
                                 kw.get("align", 16), kw.get("pool_cap"), kw.get("payload_cap"))
    assert np.array_equal(got["h2_status"], exp["h2_status"])
    assert got["n_msg"] == exp["n_msg"] and got["total"] == exp["total"]
    assert np.array_equal(got["msg_status"], exp["msg_status"])
    for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask",
              "header_size"):
        assert np.array_equal(got["msg_desc"][f], exp["msg_desc"][f]), f
    assert np.array_equal(got["payload"][:got["total"]], exp["payload"][:exp["total"]])
    return got


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_deserialize_golden_messages():
    g = golden("h2_cases.json")["messages"][0]
    stream = np.frombuffer(bytes.fromhex(g["stream_hex"]), np.uint8).copy()
    check_h2_deserialize(stream, O.h2_index(stream), align=1)
    for c in golden("h2_cases.json")["recv"]:
        raw = np.frombuffer(bytes.fromhex(c["raw_hex"]), np.uint8).copy()
        check_h2_deserialize(raw, np.array([0], np.uint64))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("S", [16384, 100])
def test_gpu_h2_roundtrip_random(S):
    rng = random.Random(S + 1)
    payload = O.fill_splitmix(1 << 20, 3, 0)
    n = 500
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 5, 126, 999, 16376, 20000, 70000])
        d[i] = (rng.randrange(0, (1 << 20) - sz), 0, sz, rng.getrandbits(32), 1,
                rng.choice([1, 2, 9]), rng.random() < .7, 0)
    h2, _ = O.h2_serialize_batch(payload, d, 1, S)
    index = O.h2_index(h2)
    check_h2_deserialize(h2, index, S=S)
    check_h2_deserialize(h2, index, S=S, align=1, payload_cap=len(h2) // 3)    # OOM tail
    check_h2_deserialize(h2, index, S=S, pool_cap=len(h2) // 2)                # pool OOM
    bad = h2.copy()
    for k in range(3, len(index), 37):                                        # corrupt headers
        bad[int(index[k]) + 3] = 6 if k % 2 else bad[int(index[k]) + 3]
        bad[int(index[k])] = 0xFF if not k % 2 else bad[int(index[k])]
    check_h2_deserialize(bad, index, S=S)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("S", [16384, 1000])
def test_gpu_h2_long_messages(S):
    """Messages of 1-4 MiB (64-256 DATA frames each at 16,384, 1,000-4,000 at
    1,000) between runs of short ones: the receive's merged layout + units
    kernel deals a long message's DATA frames out over the wave's lanes
    (ADVICE r4), and the short runs keep the per-thread walk; against the
    oracle, with a capacity cut through a long message, and the two-launch
    form (CFWS_H2_UNITS_MERGED=0) in tests/knob_parity.py."""
    rng = random.Random(S + 77)
    payload = O.fill_splitmix(5 << 20, 77, 0)
    d = []
    for i in range(90):
        if i % 9 == 4:
            sz = rng.choice([1 << 20, 3 << 20, (4 << 20) - 14, rng.randrange(1 << 20, 4 << 20)])
        else:
            sz = rng.choice([0, 5, 126, 999, 16376, 20000])
        d.append((rng.randrange(0, (5 << 20) - sz), 0, sz, rng.getrandbits(32), 1,
                  rng.choice([1, 2]), rng.random() < .8, 0))
    d = np.array(d, dtype=O.DESC_DTYPE)
    h2, _ = O.h2_serialize_batch(payload, d, 1, S)
    index = O.h2_index(h2)
    check_h2_deserialize(h2, index, S=S)
    check_h2_deserialize(h2, index, S=S, align=1, payload_cap=len(h2) // 2)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("S", [5, 13, 64])
def test_gpu_h2_deserialize_headers_across_data_frames(S):
    """DATA frames smaller than the WS header (max_frame_size 5 / 13) put a
    WS header across several DATA frames; the fused receive gathers it.
    Messages with trailing bytes after their WS frame, empty DATA frames
    and a stream cut mid-message are mixed in."""
    rng = random.Random(S * 7)
    payload = O.fill_splitmix(1 << 16, 11, 0)
    n = 60
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 1, 7, 125, 126, 300, 2000])
        d[i] = (rng.randrange(0, (1 << 16) - sz), 0, sz, rng.getrandbits(32), 1,
                rng.choice([1, 2, 9]), rng.random() < .7, 0)
    h2, _ = O.h2_serialize_batch(payload, d, 1, S)
    # an extra DATA frame (no END_STREAM) of junk in front of message 3's
    # END_STREAM frame: that message then carries bytes after its WS frame
    index = O.h2_index(h2)
    cut = int(index[len(index) // 2])
    tail = h2[cut:]
    junk = np.array([0, 0, 3, 0, 0, 0, 0, 0, 1, 0xAA, 0xBB, 0xCC], np.uint8)
    empty = np.array([0, 0, 0, 0, 0, 0, 0, 0, 1], np.uint8)
    h2 = np.concatenate([h2[:cut], empty, tail[:-4]])
    index = O.h2_index(h2)
    check_h2_deserialize(h2, index, S=S)
    check_h2_deserialize(h2, index, S=S, align=1, payload_cap=len(h2) // 4)
    # trailing junk inside a message: insert before a final DATA frame
    k = int(index[5])
    h2b = np.concatenate([h2[:k], junk, h2[k:]])
    check_h2_deserialize(h2b, O.h2_index(h2b), S=S)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("cut", [1, 2, 3])
def test_gpu_h2_stream_without_end_stream(cut):
    """Streams whose last messages never see END_STREAM: their DATA frames
    are in no message (h2_msg_apply_units_kernel hands them to the threads
    in turn as empty units). `cut` DATA frames of a 40,000-byte message's
    three are kept: 1 and 2 leave no message at all (n_messages 0) after
    a run of complete ones (3: the last message is whole)."""
    rng = random.Random(cut)
    payload = O.fill_splitmix(1 << 17, cut, 0)
    d = np.zeros(1, dtype=O.DESC_DTYPE)
    d[0] = (100, 0, 40000, rng.getrandbits(32), 1, 2, 1, 0)
    h2, _ = O.h2_serialize_batch(payload, d, 1, 16384)
    index = O.h2_index(h2)
    assert len(index) == 3
    end = int(index[cut]) if cut < 3 else len(h2)
    alone = h2[:end].copy()
    got = check_h2_deserialize(alone, O.h2_index(alone))
    assert got["n_msg"] == (1 if cut == 3 else 0)
    # the same after 300 whole messages of mixed sizes
    head, hidx = _h2_case(cut + 50, 300)
    both = np.concatenate([head, alone])
    got = check_h2_deserialize(both, O.h2_index(both))
    assert got["n_msg"] == 300 + (1 if cut == 3 else 0)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_gpu_config5_digest(idx):
    """Config 5 batches (16,376 B and 64 KiB frames, 1,024 and 65,536 of
    them): the DATA-frame stream equals the reference's byte for byte, and
    unwrap + unmask restores every payload."""
    torch, cfws = _gpu()
    from coldforce_amd import workloads as W
    g = golden("h2_digests.json")[idx]
    n, fs = g["n_frames"], g["frame_size"]
    desc = W.uniform_batch(n, fs, g["key_seed"])
    payload = torch.empty(W.round16(n * fs) + 16, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(payload, g["payload_seed"])
    offs, wtotal = W.wire_layout(desc)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
    h2 = torch.empty(cfws.h2_wrapped_bound(wire.numel(), n), dtype=torch.uint8, device="cuda")
    tot = cfws.h2_serialize(payload, cfws.desc_to_device(desc), wire, h2, g["sid"], g["max_frame"])
    torch.cuda.synchronize()
    t = int(tot.item())
    assert t == g["h2_len"]
    h = hashlib.sha256()
    for o in range(0, t, 1 << 28):
        h.update(h2[o:min(t, o + (1 << 28))].cpu().numpy().tobytes())
    assert h.hexdigest() == g["h2_sha256"]
    # DATA frame starts: k = ceil(W / S) frames per WS frame, 9-byte headers
    S = g["max_frame"]
    W_ = fs + 14 if fs > 65535 else fs + 8
    k = -(-W_ // S)
    starts = np.concatenate([f * (W_ + 9 * k) + np.arange(k) * (S + 9) for f in range(n)]) \
        if n <= 1024 else None
    if starts is None:
        per = (W_ + 9 * k) * np.arange(n, dtype=np.uint64)
        starts = (per[:, None] + (np.arange(k, dtype=np.uint64) * (S + 9))[None, :]).reshape(-1)
    idx_t = torch.from_numpy(starts.astype(np.int64)).cuda()
    pool = torch.empty(t, dtype=torch.uint8, device="cuda")
    back = torch.empty(n * fs + 64, dtype=torch.uint8, device="cuda")
    st, md, ms, ptot, m = cfws.h2_deserialize(h2, t, idx_t, pool, back, S, align=1)
    torch.cuda.synchronize()
    assert m == n and int(ptot.item()) == n * fs
    assert bool((st == 0).all()) and bool((ms == 0).all())
    assert torch.equal(back[:n * fs], payload[:n * fs])


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_roundtrip_600k_frames():
    """600,000 small WS frames, one DATA frame each: the plans run with more
    than 2,048 blocks (a scan launch of their own for the block sums in the
    H2 plans; the single-pass look-back in the WS deserialize plan the pool
    overflow's general form runs, with per-message ends). Send and receive
    vs the oracle, with the pool holding everything and half of it."""
    rng = np.random.default_rng(600)
    n = 600_000
    payload = O.fill_splitmix(1 << 20, 600, 0)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    sz = rng.choice(np.array([0, 1, 7, 60, 125, 126, 200], np.uint64), n)
    d["payload_off"] = rng.integers(0, (1 << 20) - 256, n).astype(np.uint64)
    d["payload_size"] = sz
    d["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    d["fin"], d["opcode"], d["mask"] = 1, 2, (rng.random(n) < .7).astype(np.uint8)
    exp, _ = O.h2_serialize_batch(payload, d, 3, 16384)
    got, t = gpu_h2_serialize(payload, d, 3, 16384)
    assert t == len(exp) and np.array_equal(got, exp)
    index = O.h2_index(exp)
    assert len(index) == n
    check_h2_deserialize(exp, index, align=1)
    check_h2_deserialize(exp, index, align=1, pool_cap=len(exp) // 2)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_deserialize_two_threads():
    """The receive plan hands its message count to the host through mapped
    host words, one pair per host thread: two threads decoding different
    batches on their own streams at once each get their own counts and
    payloads (ctypes releases the GIL during the call)."""
    import threading
    torch, cfws = _gpu()
    cases = []
    for seed, n in ((11, 300), (12, 700)):
        rng = random.Random(seed)
        payload = O.fill_splitmix(1 << 20, seed, 0)
        d = np.zeros(n, dtype=O.DESC_DTYPE)
        for i in range(n):
            sz = rng.choice([0, 7, 126, 1000, 16376, 40000])
            d[i] = (rng.randrange(0, (1 << 20) - sz), 0, sz, rng.getrandbits(32), 1, 2,
                    rng.random() < .5, 0)
        h2, _ = O.h2_serialize_batch(payload, d, 1, 16384)
        index = O.h2_index(h2)
        exp = O.h2_deserialize_batch(h2, index, 16384, O.DEFAULT_MAX_PAYLOAD, 16, None, None)
        h = torch.from_numpy(np.concatenate([h2, np.zeros(16, np.uint8)])).cuda()
        idx = torch.from_numpy(index.astype(np.int64)).cuda()
        pool = torch.empty(len(h2) + 16, dtype=torch.uint8, device="cuda")
        pay = torch.empty(len(h2) + 16 * len(index) + 16, dtype=torch.uint8, device="cuda")
        cases.append((h, len(h2), idx, pool, pay, exp, torch.cuda.Stream()))
    torch.cuda.synchronize()
    errors = []

    def run(case):
        h, size, idx, pool, pay, exp, s = case
        try:
            for _ in range(8):
                st, md, ms, tot, m = cfws.h2_deserialize(h, size, idx, pool, pay, stream=s)
                s.synchronize()
                assert m == exp["n_msg"] and int(tot.item()) == exp["total"]
                assert np.array_equal(pay[:exp["total"]].cpu().numpy(), exp["payload"][:exp["total"]])
        except Exception as e:          # reported from the main thread
            errors.append(e)

    ts = [threading.Thread(target=run, args=(c,)) for c in cases]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def _h2_case(seed, n, sizes=(0, 7, 126, 1000, 16376, 40000)):
    rng = random.Random(seed)
    payload = O.fill_splitmix(1 << 20, seed, 0)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice(sizes)
        d[i] = (rng.randrange(0, (1 << 20) - sz), 0, sz, rng.getrandbits(32), 1, 2,
                rng.random() < .5, 0)
    h2, _ = O.h2_serialize_batch(payload, d, 1, 16384)
    return h2, O.h2_index(h2)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("pool_div", [None, 2, 5])
def test_gpu_h2_rows_past_message_count_are_empty(pool_div):
    """Every message row past n_messages is an empty entry (no payload, no
    header, MORE_DATA), whether the fused form ran or the pool overflowed and the
    general form redid the call with fewer messages; the payloads still
    equal the oracle's (the fused payload pass stores nothing on overflow)."""
    torch, cfws = _gpu()
    h2, index = _h2_case(21, 400)
    pool_cap = None if pool_div is None else len(h2) // pool_div
    exp = O.h2_deserialize_batch(h2, index, 16384, O.DEFAULT_MAX_PAYLOAD, 16, pool_cap, None)
    h = torch.from_numpy(np.concatenate([h2, np.zeros(16, np.uint8)])).cuda()
    idx = torch.from_numpy(index.astype(np.int64)).cuda()
    pool = torch.empty(len(h2) if pool_cap is None else pool_cap, dtype=torch.uint8, device="cuda")
    pay = torch.full((len(h2) + 16 * len(index) + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    st, md, ms, tot, m = cfws.h2_deserialize(h, len(h2), idx, pool, pay, all_rows=True)
    torch.cuda.synchronize()
    assert m == exp["n_msg"] and int(tot.item()) == exp["total"]
    assert m < len(index)
    assert np.array_equal(pay[:exp["total"]].cpu().numpy(), exp["payload"][:exp["total"]])
    assert np.array_equal(ms[:m].cpu().numpy(), exp["msg_status"])
    # empty entries: no payload, no header; payload_off is the layout's
    # position (the end of the messages' payloads in the fused form)
    rest = cfws.desc_from_device(md[m:])
    for f in ("wire_off", "payload_size", "mask_key", "fin", "opcode", "mask", "header_size"):
        assert not rest[f].any(), f
    assert bool((ms[m:] == O.PARSE_MORE_DATA).all())


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_deserialize_thread_churn():
    """Short-lived host threads, one call each, three at a time: each thread
    borrows the receive handoff (mapped count words + event) for the stream's
    device and hands it back when it exits, so later threads reuse it. Every
    call gets its own counts and payloads."""
    import threading
    torch, cfws = _gpu()
    h2, index = _h2_case(31, 300)
    exp = O.h2_deserialize_batch(h2, index, 16384, O.DEFAULT_MAX_PAYLOAD, 16, None, None)
    h = torch.from_numpy(np.concatenate([h2, np.zeros(16, np.uint8)])).cuda()
    idx = torch.from_numpy(index.astype(np.int64)).cuda()
    bufs = [(torch.empty(len(h2) + 16, dtype=torch.uint8, device="cuda"),
             torch.empty(len(h2) + 16 * len(index) + 16, dtype=torch.uint8, device="cuda"),
             torch.cuda.Stream()) for _ in range(3)]
    torch.cuda.synchronize()
    errors = []

    def run(k):
        pool, pay, s = bufs[k]
        try:
            st, md, ms, tot, m = cfws.h2_deserialize(h, len(h2), idx, pool, pay, stream=s)
            s.synchronize()
            assert m == exp["n_msg"] and int(tot.item()) == exp["total"]
            assert np.array_equal(pay[:exp["total"]].cpu().numpy(), exp["payload"][:exp["total"]])
        except Exception as e:          # reported from the main thread
            errors.append(e)

    for _ in range(8):
        ts = [threading.Thread(target=run, args=(k,)) for k in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errors, errors


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
def test_gpu_h2_deserialize_stream_on_other_device():
    """The receive handoff is keyed by the STREAM's device, not the thread's
    current one: a call whose stream and buffers live on device 1 while
    device 0 is current decodes correctly (needs two GPUs)."""
    torch, cfws = _gpu()
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    h2, index = _h2_case(41, 200)
    exp = O.h2_deserialize_batch(h2, index, 16384, O.DEFAULT_MAX_PAYLOAD, 16, None, None)
    dev = torch.device("cuda", 1)
    h = torch.from_numpy(np.concatenate([h2, np.zeros(16, np.uint8)])).to(dev)
    idx = torch.from_numpy(index.astype(np.int64)).to(dev)
    pool = torch.empty(len(h2) + 16, dtype=torch.uint8, device=dev)
    pay = torch.empty(len(h2) + 16 * len(index) + 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_device(0)
    for _ in range(2):
        st, md, ms, tot, m = cfws.h2_deserialize(h, len(h2), idx, pool, pay, stream=s)
        s.synchronize()
        assert m == exp["n_msg"] and int(tot.item()) == exp["total"]
        assert np.array_equal(pay[:exp["total"]].cpu().numpy(), exp["payload"][:exp["total"]])


# ---- the reference's own stream code on multi-DATA-frame WS frames ---------------
# tests/golden/h2_echo_digests.json: the DATA frames the stock echo pair
# (oracle/_ref/ws_echo_stock: co_http2_stream_send_ws_frame ->
# co_http2_stream_send_data, co_http2_stream.c:933-1013, and the peer's
# pooling, :550-608) put on the wire for TEXT frames of 16,376 B (one DATA
# frame), 16,377 B (16,384 + 1), 40,000 B (2 x 16,384 + 7,240) and 65,536 B
# (4 x 16,384 + 14), client-masked after srandom(seed), echoed unmasked.

def _echo_batch(case, side):
    """The WS frames one side of the echo sent: frame k is TEXT, fin, with
    payload 'a' + (j + k) % 26 (oracle/ws_echo.c fill_frame), masked with
    the k-th key of srandom(seed) on the client side."""
    from echo_util import frame_text
    n, fs = case["frames"], case["payload"]
    arena = np.frombuffer(b"".join(frame_text(k, fs) for k in range(n)), np.uint8).copy()
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * fs
    d["payload_size"], d["fin"], d["opcode"] = fs, 1, case["opcode"]
    if case[side]["mask"]:
        d["mask"] = 1
        d["mask_key"] = O.keys(case["seed"], n)
    return arena, d


def _echo_cases():
    return golden("h2_echo_digests.json")


@pytest.mark.parametrize("i", range(4))
def test_oracle_matches_stock_h2_echo_golden(i):
    """The restatement's DATA split (cfws_oracle.c) gives the bytes the
    reference's stream code put on the wire, both directions, and its
    receive pools them back into the payloads."""
    case = _echo_cases()[i]
    for side in ("client", "server"):
        g = case[side]
        arena, d = _echo_batch(case, side)
        h2, _ = O.h2_serialize_batch(arena, d, case["sid"], case["max_frame"])
        assert len(h2) == g["data_len"] and sha(h2) == g["data_sha256"], side
        idx = O.h2_index(h2)
        assert len(idx) == g["data_frames"]
        assert [int(h2[p]) << 16 | int(h2[p + 1]) << 8 | int(h2[p + 2]) for p in idx[:len(g["split"])]] \
            == g["split"]
        r = O.h2_deserialize_batch(h2, idx, case["max_frame"], align=1, payload_capacity=len(arena))
        assert r["n_msg"] == case["frames"] and (r["msg_status"][:r["n_msg"]] == 0).all()
        assert np.array_equal(r["payload"][:len(arena)], arena)


@pytest.mark.parametrize("i", range(4))
def test_stock_h2_echo_reproduces_golden(i, tmp_path):
    """Re-runs the stock echo pair (the reference's http2 + ws_http2 code
    compiled in place) and checks its capture against the fixture."""
    from echo_util import available, h2_data_frames, run_echo
    if not available("stock"):
        pytest.skip("oracle/_ref/ws_echo_stock not built")
    case = _echo_cases()[i]
    r = run_echo("stock", "h2", case["frames"], case["payload"], window=case["window"], seed=case["seed"],
                 capture_dir=str(tmp_path))
    assert r["client_rc"] == 0 and r["client"]["received"] == case["frames"] and r["client"]["bad_echo"] == 0
    for side in ("client", "server"):
        with open(r["capture"][side], "rb") as f:
            data = h2_data_frames(f.read(), preface=side == "client")
        raw = b"".join(x for _, x in data)
        assert sha(raw) == case[side]["data_sha256"], side
        assert sum(1 for fl, _ in data if fl & 1) == case[side]["end_stream"] == case["frames"]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("i", range(4))
def test_gpu_h2_matches_stock_h2_echo(i):
    """cfws_h2_serialize_batch on the echo's frames gives the DATA frames
    the reference's stream code sent (split, END_STREAM on the last frame of
    each WS frame, stream 1), both directions; cfws_h2_deserialize_batch
    pools them back into the payloads."""
    torch, cfws = _gpu()
    case = _echo_cases()[i]
    for side in ("client", "server"):
        g = case[side]
        arena, d = _echo_batch(case, side)
        got, t = gpu_h2_serialize(arena, d, case["sid"], case["max_frame"])
        assert t == g["data_len"] and sha(got) == g["data_sha256"], side
        idx = O.h2_index(got)
        h = torch.from_numpy(np.concatenate([got, np.zeros(16, np.uint8)])).cuda()
        idx_t = torch.from_numpy(idx.astype(np.int64)).cuda()
        pool = torch.empty(t + 16, dtype=torch.uint8, device="cuda")
        pay = torch.empty(len(arena) + 16 * len(idx) + 16, dtype=torch.uint8, device="cuda")
        st, md, ms, tot, m = cfws.h2_deserialize(h, t, idx_t, pool, pay, case["max_frame"], align=1)
        torch.cuda.synchronize()
        assert m == case["frames"] and bool((st == 0).all()) and bool((ms == 0).all())
        assert int(tot.item()) == len(arena)
        assert np.array_equal(pay[:len(arena)].cpu().numpy(), arena)
