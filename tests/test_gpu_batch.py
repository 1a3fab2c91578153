"""GPU parity: the MI355X batch codec (libcfws.so, include/cfws.h) against the
oracle (CPU restatement, pinned to the reference) and against digests the
reference codec itself produced (tests/golden/batch_digests.json).
Bit-exact everywhere: this is byte work."""
import hashlib
import random

import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

SIZES = [0, 1, 3, 4, 5, 15, 16, 17, 124, 125, 126, 127, 128, 1000, 4095, 4096, 4097,
         65535, 65536, 65537, 1 << 20]


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()
    return torch.device("cuda", 0)


def sha(a) -> str:
    return hashlib.sha256(a.tobytes() if hasattr(a, "tobytes") else a).hexdigest()


def gpu_serialize(payload: np.ndarray, desc: np.ndarray, slack: int = 0, capacity=None,
                  plan_execute=False):
    pay = torch.from_numpy(payload if payload.size else np.zeros(16, np.uint8)).cuda()
    d_t = cfws.desc_to_device(desc)
    _, total = W.wire_layout(desc)
    cap = W.round16(total) + slack if capacity is None else capacity
    wire = torch.full((max(cap, 16),), 0xEE, dtype=torch.uint8, device="cuda")
    if plan_execute:
        ws = cfws.workspace(len(desc), cap)
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        cfws.serialize_plan(d_t, cap, tot, ws)
        cfws.serialize_execute(pay, d_t, wire, ws, cap)
    else:
        tot = cfws.serialize(pay, d_t, wire[:cap] if cap else wire[:0])
    torch.cuda.synchronize()
    return wire.cpu().numpy(), cfws.desc_from_device(d_t), int(tot.item()), total


def random_desc(rng, n, payload_len, sizes=None, aligned=False):
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice(sizes) if sizes else rng.randrange(0, 3000)
        sz = min(sz, payload_len)
        off = rng.randrange(0, payload_len - sz + 1)
        if aligned:
            off -= off % 16
        d[i]["payload_off"] = off
        d[i]["payload_size"] = sz
        d[i]["fin"] = rng.random() < 0.7
        d[i]["opcode"] = rng.randrange(256) if rng.random() < 0.1 else rng.choice([0, 1, 2, 8, 9, 10])
        d[i]["mask"] = rng.random() < 0.6
        d[i]["mask_key"] = rng.getrandbits(32) if d[i]["mask"] else 0
    return d


def check_serialize(payload, desc, **kw):
    wire, d_out, tot, total = gpu_serialize(payload, desc, **kw)
    exp, d_exp = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    assert tot == total == len(exp)
    assert np.array_equal(d_out["wire_off"], d_exp["wire_off"])
    assert np.array_equal(d_out["header_size"], d_exp["header_size"])
    bad = np.nonzero(wire[:total] != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    return wire, total


def test_serialize_boundary_sizes():
    rng = random.Random(1)
    payload = O.fill_splitmix(3 << 20, 0x1234, 0)
    d = []
    for n in SIZES:
        for mask in (False, True):
            for fin, op in ((True, 2), (False, 0), (True, 0x7F), (False, 0xFF)):
                d.append((rng.randrange(0, (3 << 20) - n), n, fin, op, mask, rng.getrandbits(32)))
    desc = np.zeros(len(d), dtype=cfws.DESC_DTYPE)
    for i, (off, n, fin, op, mask, key) in enumerate(d):
        desc[i] = (off, 0, n, key if mask else 0, fin, op, mask, 0)
    wire, total = check_serialize(payload, desc)
    # bytes past the total inside the rounded-up capacity are written as zero
    assert not wire[total:W.round16(total)].any()


@pytest.mark.parametrize("seed", [2, 3, 4])
def test_serialize_random_mix(seed):
    rng = random.Random(seed)
    payload = O.fill_splitmix(1 << 20, seed, 0)
    desc = random_desc(rng, 4000, 1 << 20, aligned=seed == 4)
    check_serialize(payload, desc, plan_execute=seed == 3)


def test_serialize_tiny_frames_dense():
    # > 1024 frames per 16 KiB tile (2-6 byte frames): exercises the
    # global-search path of the tile scheduler.
    rng = random.Random(9)
    payload = O.fill_splitmix(4096, 9, 0)
    desc = random_desc(rng, 20000, 4096, sizes=[0, 0, 1, 2, 3])
    check_serialize(payload, desc)


def test_serialize_keys_from_random():
    # Keys drawn by cfws_draw_mask_keys after srandom(s) == reference key stream.
    for seed, ks in golden("keys.json").items():
        got = cfws.draw_mask_keys(len(ks), seed=int(seed))
        assert [int.from_bytes(bytes.fromhex(k), "little") for k in ks] == list(map(int, got))


def test_serialize_capacity_truncation():
    rng = random.Random(5)
    payload = O.fill_splitmix(1 << 16, 5, 0)
    desc = random_desc(rng, 50, 1 << 16)
    _, total = W.wire_layout(desc)
    cap = total // 2 + 3
    wire, _, tot, _ = gpu_serialize(payload, desc, capacity=cap)
    exp, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    assert tot == total                       # unclamped total is reported
    assert np.array_equal(wire[:cap], exp[:cap])
    assert (wire[cap:] == 0xEE).all()         # nothing written past capacity


def gpu_deserialize(wire: np.ndarray, starts: np.ndarray, align=16, capacity=None,
                    max_payload=O.DEFAULT_MAX_PAYLOAD, plan_execute=False, flags=0):
    w = torch.from_numpy(np.concatenate([wire, np.zeros(16, np.uint8)])).cuda()
    idx = torch.from_numpy(starts.astype(np.int64)).cuda()
    cap = capacity if capacity is not None else len(wire) + 16 * len(starts) + 16
    out = torch.full((max(cap, 16),), 0xEE, dtype=torch.uint8, device="cuda")
    if plan_execute:
        n = len(starts)
        ws = cfws.workspace(n, cap)
        d_t = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        st_t = torch.empty(n, dtype=torch.int32, device="cuda")
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        cfws.deserialize_plan(w, len(wire), idx, d_t, st_t, cap, tot, ws, max_payload, align,
                              flags=flags)
        cfws.deserialize_execute(w, d_t, st_t, out, ws, cap, flags=flags)
    else:
        d_t, st_t, tot = cfws.deserialize(w, len(wire), idx, out[:cap], max_payload=max_payload,
                                          align=align, flags=flags)
    torch.cuda.synchronize()
    return out.cpu().numpy(), cfws.desc_from_device(d_t), st_t.cpu().numpy(), int(tot.item())


def check_deserialize(wire, starts, **kw):
    out, d, st, tot = gpu_deserialize(wire, starts, **kw)
    cap = kw.get("capacity") or len(wire) + 16 * len(starts) + 16
    e_out, e_d, e_st, e_tot = O.deserialize_batch(wire, starts, align=kw.get("align", 16),
                                                  max_payload=kw.get("max_payload",
                                                                     O.DEFAULT_MAX_PAYLOAD),
                                                  capacity=cap, flags=kw.get("flags", 0))
    assert tot == e_tot
    assert np.array_equal(st, e_st)
    for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask",
              "header_size"):
        assert np.array_equal(d[f], e_d[f]), f
    bad = np.nonzero(out[:tot] != e_out[:tot])[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    return out, d, st, tot


def wire_stream(rng, n, sizes=None):
    frames, payloads = [], []
    for _ in range(n):
        sz = rng.choice(sizes) if sizes else rng.randrange(0, 3000)
        p = rng.randbytes(sz)
        payloads.append(p)
        frames.append(O.serialize_keyed(rng.random() < .7, rng.randrange(16), rng.random() < .6,
                                        rng.getrandbits(32), p))
    return np.frombuffer(b"".join(frames), dtype=np.uint8).copy(), payloads


@pytest.mark.parametrize("align", [1, 16, 64, 4096])
def test_deserialize_random_stream(align):
    rng = random.Random(align)
    wire, payloads = wire_stream(rng, 3000, sizes=SIZES[:-1] + [rng.randrange(70000)])
    starts, consumed = O.index_frames(wire, 10000)
    assert consumed == len(wire)
    cap = len(wire) + align * (len(starts) + 1)
    out, d, st, tot = check_deserialize(wire, starts, align=align, capacity=cap,
                                        plan_execute=align == 64)
    assert (st == 0).all()
    for i, p in enumerate(payloads[:200]):
        o = int(d["payload_off"][i])
        assert out[o:o + len(p)].tobytes() == p


@pytest.mark.parametrize("plan_execute", [False, True])
def test_deserialize_reassemble(plan_execute):
    """Fragmented messages with control frames interleaved (RFC 6455 5.4):
    data payloads come out packed in stream order, controls after them."""
    rng = random.Random(21 + plan_execute)
    frames = []
    for m in range(400):
        nfrag = rng.randrange(1, 6)
        for j in range(nfrag):
            op = (rng.choice([1, 2]) if j == 0 else 0)
            p = rng.randbytes(rng.choice([0, 1, 17, 125, 126, 4000, 70000]))
            frames.append(O.serialize_keyed(j == nfrag - 1, op, rng.random() < .8,
                                            rng.getrandbits(32), p))
            if rng.random() < 0.2:
                frames.append(O.serialize_keyed(True, rng.choice([8, 9, 10]), True,
                                                rng.getrandbits(32), rng.randbytes(rng.randrange(126))))
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    starts, _ = O.index_frames(wire, 100000)
    check_deserialize(wire, starts, flags=1, plan_execute=plan_execute)
    # errors and a tight capacity under reassembly
    wire[int(starts[7])] |= 0x20
    check_deserialize(wire, starts, flags=1, capacity=len(wire) // 3)


@pytest.mark.parametrize("shift", [0, 3, 13])
def test_plan_any_wire_alignment(shift):
    """The receive plan reads each header with one unaligned 16-byte load
    (deserialize_plan_single_kernel, > 2,048 plan blocks), so it takes a wire
    at any byte address: 600,000 frames of 0-300 bytes (7-bit and 16-bit
    lengths, masked and not) planned from a wire shifted by `shift` bytes,
    with invalid headers and a truncated last frame, against the oracle's
    descriptors, statuses and total."""
    rng = np.random.default_rng(shift + 40)
    n = 600_000
    payload = O.fill_splitmix(1 << 16, shift, 0)
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    desc["payload_size"] = rng.integers(0, 301, n).astype(np.uint64)
    desc["payload_off"] = rng.integers(0, (1 << 16) - 400, n).astype(np.uint64)
    desc["fin"] = 1
    desc["opcode"] = rng.choice([1, 2, 9], n).astype(np.uint8)
    desc["mask"] = (rng.random(n) < 0.6).astype(np.uint8)
    desc["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * desc["mask"]
    exp_wire, d2 = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    offs = d2["wire_off"].astype(np.uint64)
    w = exp_wire.copy()
    w[offs[rng.choice(n - 1, 100, replace=False)].astype(np.int64)] |= 0x20      # an RSV bit -> INVALID_FRAME
    w = w[:len(w) - 2]                                                          # MORE_DATA at the end
    buf = torch.from_numpy(np.concatenate([np.zeros(shift, np.uint8), w, np.zeros(16, np.uint8)])).cuda()
    wt = buf[shift:]
    assert (wt.data_ptr() - buf.data_ptr()) == shift
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    cap = len(w) + 16 * n
    ws = cfws.workspace(n, cap)
    d_t = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    st_t = torch.empty(n, dtype=torch.int32, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cfws.deserialize_plan(wt, len(w), idx, d_t, st_t, cap, tot, ws, align=16)
    torch.cuda.synchronize()
    _, e_d, e_st, e_tot = O.deserialize_batch(w, offs, align=16, capacity=cap)
    assert int(tot.item()) == e_tot
    st = st_t.cpu().numpy()
    assert np.array_equal(st, e_st) and (st == O.ERROR_INVALID_FRAME).sum() >= 100
    d = cfws.desc_from_device(d_t)
    for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask", "header_size"):
        assert np.array_equal(d[f], e_d[f]), f


def test_deserialize_error_frames():
    rng = random.Random(7)
    wire, _ = wire_stream(rng, 200)
    starts, _ = O.index_frames(wire, 1000)
    # corrupt some headers, add truncated / out-of-range starts, vary limits
    wire = wire.copy()
    for i in range(0, len(starts), 17):
        wire[int(starts[i])] |= 0x40           # RSV2 -> INVALID_FRAME
    extra = np.array([len(wire) - 1, len(wire), len(wire) + 7, int(starts[5]) + 1], dtype=np.uint64)
    starts2 = np.concatenate([starts, extra])
    check_deserialize(wire, starts2)
    check_deserialize(wire, starts2, max_payload=1000)
    check_deserialize(wire, starts2, capacity=10000)   # OUT_OF_MEMORY from some frame on


def test_deserialize_golden_cases():
    # every fixture case that is small enough, through the batch path
    for c in golden("deserialize_cases.json"):
        if c["wire_hex"] is None:
            continue
        raw = np.frombuffer(bytes.fromhex(c["wire_hex"]), dtype=np.uint8).copy()
        out, d, st, tot = gpu_deserialize(raw, np.array([c["index"]], np.uint64), align=1,
                                          max_payload=c["max_payload"])
        exp_rc = c["rc"]
        if len(raw) - c["index"] < 2:
            exp_rc = O.PARSE_MORE_DATA
        assert st[0] == exp_rc, c["name"]
        if exp_rc == 0:
            assert int(d["payload_size"][0]) == c["payload_size"]
            if c["payload_hex"] is not None:
                assert out[:c["payload_size"]].tobytes() + b"\0" == bytes.fromhex(c["payload_hex"])
        if exp_rc in (0, O.ERROR_INVALID_FRAME):
            assert bool(d["fin"][0]) == c["fin"] and int(d["opcode"][0]) == c["opcode"]


def test_config2_reduced_digest():
    g = golden("batch_digests.json")[0]
    _roundtrip_digest(g)


def test_config2_full_size_digest():
    """65,536 x 64 KiB (BASELINE configs[1]) at full size: the wire arena is
    bit-identical to the reference's serialize output (SHA-256 of 4.0009 GiB)
    and deserialize restores every payload byte."""
    g = golden("batch_digests.json")[2]
    _roundtrip_digest(g, full=True)


def _sha_device(t: "torch.Tensor", n: int) -> str:
    h = hashlib.sha256()
    step = 1 << 28
    for o in range(0, n, step):
        h.update(t[o:min(n, o + step)].cpu().numpy().tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("which", [0, 1, 2, 3, 4, 5],
                         ids=["4M_x_1KiB_text", "16M_x_256B_binary", "2M_x_2KiB_binary",
                              "1398101_x_3KiB_binary", "1198372_x_3584B_text", "8M_x_512B_binary"])
def test_small_frame_reference_digests(which):
    """The small-frame batches the bench quotes (4,194,304 x 1 KiB TEXT,
    16,777,216 x 256 B BINARY, and the in-region send's range: 2,097,152 x
    2 KiB, 1,398,101 x 3 KiB and 1,198,372 x 3,584 B -- the bound itself --
    every one 4 GiB of payload at the bench's seeds) through the bench's own
    calls: serialize plan + execute (single-pass look-back plan, in-region
    send edges) and deserialize plan + execute at 16-byte slots, then the
    slot and scatter receives. The wire's SHA-256 equals the reference's
    co_ws_frame_serialize output
    (co_ws_frame.c:21-119, compiled in place, tests/golden/make_golden.py
    small_batch_digest), and the unmasked payloads' SHA-256 equals what the
    reference's co_ws_frame_deserialize walk (co_ws_frame.c:121-247) returned
    from that wire."""
    g = golden("small_batch_digests.json")[which]
    n, fs = g["n_frames"], g["frame_size"]
    desc = W.uniform_batch(n, fs, g["key_seed"], opcode=g["opcode"])
    offs, total = W.wire_layout(desc)
    assert total == g["wire_len"]
    payload = torch.empty(n * fs, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(payload, g["payload_seed"])
    d_t = cfws.desc_to_device(desc)
    wire = torch.full((W.round16(total),), 0xEE, dtype=torch.uint8, device="cuda")
    ws = cfws.workspace(n, wire.numel())
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cfws.serialize_plan(d_t, wire.numel(), tot, ws)
    cfws.serialize_execute(payload, d_t, wire, ws)
    torch.cuda.synchronize()
    assert tot.item() == total
    assert _sha_device(wire, total) == g["wire_sha256"]
    del ws
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    back = torch.full((n * fs + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    desc_de = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    status = torch.full((n,), 99, dtype=torch.int32, device="cuda")
    ws = cfws.workspace(n, back.numel())
    ptot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cfws.deserialize_plan(wire, total, idx, desc_de, status, back.numel(), ptot, ws, align=16)
    cfws.deserialize_execute(wire, desc_de, status, back, ws)
    torch.cuda.synchronize()
    assert ptot.item() == n * fs and bool((status == 0).all())
    assert _sha_device(back, n * fs) == g["payload_sha256"]
    assert torch.equal(back[:n * fs], payload)
    # the one-call form (256 B frames: the fused plan + copy kernel)
    back.fill_(0xEE)
    status.fill_(99)
    _, st2, ptot2 = cfws.deserialize(wire, total, idx, back, desc_de, status, ws, align=16)
    torch.cuda.synchronize()
    assert ptot2.item() == n * fs and bool((st2 == 0).all())
    assert _sha_device(back, n * fs) == g["payload_sha256"]
    # cfws_deserialize_slots at slots of fs bytes: the same arena (every fs
    # here is a multiple of 16); up to 8,160 B the window kernel
    back.fill_(0xEE)
    status.fill_(99)
    _, st3, ptot3 = cfws.deserialize_slots(wire, total, idx, back, fs, desc_de, status)
    torch.cuda.synchronize()
    assert ptot3.item() == n * fs and bool((st3 == 0).all())
    assert _sha_device(back, n * fs) == g["payload_sha256"]
    # cfws_deserialize_scatter: frame i to slot (i + h) mod n, so no frame
    # lands where slot order puts it; rolled back, the payloads' SHA-256
    h = n // 2 + 1
    dst = ((torch.arange(n, dtype=torch.int64, device="cuda") + h) % n) * fs
    back.fill_(0xEE)
    status.fill_(99)
    _, st4 = cfws.deserialize_scatter(wire, total, idx, dst, back, fs, desc_de, status)
    torch.cuda.synchronize()
    assert bool((st4 == 0).all())
    rolled = torch.roll(back[:n * fs].view(n, fs), shifts=-h, dims=0).reshape(-1)
    assert _sha_device(rolled, n * fs) == g["payload_sha256"]
    del rolled
    # the compact forms: the slot and scatter receives writing 8-byte
    # cfws_frame_info_t entries (the payloads compared on the device with
    # the arena the digest above pinned) ...
    info = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    for scatter in (False, True):
        back.fill_(0xEE)
        info.fill_(0xEE)
        if scatter:
            cfws.deserialize_scatter_info(wire, total, idx, dst, back, fs, info)
        else:
            cfws.deserialize_slots_info(wire, total, idx, back, fs, info)
        torch.cuda.synchronize()
        got = back[:n * fs].view(n, fs)
        if scatter:
            got = torch.roll(got, shifts=-h, dims=0)
        assert torch.equal(got.reshape(-1), payload)
        fi = info.view(torch.int64).view(-1)
        exp = fs | 1 << 32 | g["opcode"] << 40          # payload_size, fin, opcode, status 0
        assert bool((fi == exp).all())
    del info
    # ... and the uniform send (payload + one key per frame, no plan): the
    # wire equals the one whose digest is checked above
    keys_t = torch.from_numpy(desc["mask_key"].view(np.int32).copy()).cuda()
    wire2 = torch.full_like(wire, 0xEE)
    tot_u = torch.zeros(1, dtype=torch.int64, device="cuda")
    cfws.serialize_uniform(payload, keys_t, n, fs, wire2, fin=True, opcode=g["opcode"], mask=True, total_t=tot_u)
    torch.cuda.synchronize()
    assert tot_u.item() == total and torch.equal(wire2, wire)


def _roundtrip_digest(g, full=False):
    n, fs = g["n_frames"], g["frame_size"]
    desc = W.uniform_batch(n, fs, g["key_seed"])
    offs, total = W.wire_layout(desc)
    assert total == g["wire_len"]
    payload = torch.empty(n * fs, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(payload, g["payload_seed"])
    d_t = cfws.desc_to_device(desc)
    wire = torch.empty(W.round16(total), dtype=torch.uint8, device="cuda")
    tot = cfws.serialize(payload, d_t, wire)
    torch.cuda.synchronize()
    assert tot.item() == total
    h = hashlib.sha256()
    step = 1 << 28
    for o in range(0, total, step):
        h.update(wire[o:min(total, o + step)].cpu().numpy().tobytes())
    assert h.hexdigest() == g["wire_sha256"]
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    back = torch.empty(n * fs, dtype=torch.uint8, device="cuda")
    _, st, ptot = cfws.deserialize(wire, total, idx, back, align=16)
    torch.cuda.synchronize()
    assert ptot.item() == n * fs and bool((st == 0).all())
    assert torch.equal(back, payload)
    if not full:
        assert sha(back.cpu().numpy()) == g["payload_sha256"]


def test_fill_splitmix_matches_oracle():
    for n, base in ((1000, 0), (4096, 8), (77777, 1 << 20)):
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        cfws.fill_splitmix(t, 0xABCDEF, base)
        assert np.array_equal(t.cpu().numpy(), O.fill_splitmix(n, 0xABCDEF, base))


@pytest.mark.parametrize("n", [1, 5, 16, 17, 1000, 65536, 65550, 1 << 20])
def test_xor_mask(n):
    src = torch.randint(0, 256, (n + 32,), dtype=torch.uint8, device="cuda")
    for phase in range(4):
        for so in (0, 3):
            dst = torch.zeros(n + 32, dtype=torch.uint8, device="cuda")
            cfws.xor_mask(src[so:], dst[so:], n, 0xA1B2C3D4, phase)
            s = src.cpu().numpy()[so:so + n]
            kb = np.array([0xD4, 0xC3, 0xB2, 0xA1], np.uint8)
            exp = s ^ kb[(np.arange(n) + phase) % 4]
            assert np.array_equal(dst.cpu().numpy()[so:so + n], exp)


@pytest.mark.parametrize("seed", [21, 22])
def test_small_frame_regions_both_forms(seed):
    """Runs of 30-80-byte frames put 40-130 frames into a 4 KiB output region,
    on both sides of the 64-frame line between general_region's lane-parallel
    form and its per-chunk search; occasional 5,000-byte frames add one- and
    two-frame regions. Serialize, then deserialize the same wire packed
    (align 1), aligned (16) and reassembled, against the oracle."""
    rng = random.Random(seed)
    n = 6000
    payload = O.fill_splitmix(1 << 20, seed, 0)
    sizes = [rng.randrange(30, 80) for _ in range(n)]
    for i in range(0, n, 97):
        sizes[i] = 5000
    desc = random_desc(rng, n, 1 << 20, sizes=None)
    desc["payload_size"] = sizes
    desc["payload_off"] = [rng.randrange(0, (1 << 20) - s) for s in sizes]
    desc["opcode"] = [rng.choice([0, 1, 2, 8, 9, 10]) for _ in range(n)]    # no RSV bits
    wire, total = check_serialize(payload, desc)
    w = wire[:total].copy()
    starts, consumed = O.index_frames(w, n + 1)
    assert consumed == total and len(starts) == n
    for align in (1, 16):
        check_deserialize(w, starts, align=align)
    check_deserialize(w, starts, flags=cfws.DESERIALIZE_REASSEMBLE)


@pytest.mark.parametrize("fs", [1000, 1024, 2048])
def test_many_small_frames_round_trip(fs):
    """Config 1's frame size in a batch of 128 MiB: the paths small frames
    take on a large grid (edge workgroups spread through the grid,
    register-limited residency, plans over > 2,048 blocks with the block-sum
    scan) against the oracle, then deserialize back at 16-byte slots."""
    n = (128 << 20) // fs
    payload = O.fill_splitmix(n * fs, 0x5EED0001 + fs, 0)
    desc = W.uniform_batch(n, fs, 1, opcode=cfws.OPCODE_TEXT)
    wire, total = check_serialize(payload, desc)
    offs, _ = W.wire_layout(desc)
    slot = W.round16(fs)
    w_t = torch.from_numpy(wire[:W.round16(total)].copy()).cuda()
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    back = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    _, st, ptot = cfws.deserialize(w_t, total, idx, back, align=16)
    torch.cuda.synchronize()
    assert ptot.item() == n * slot and bool((st == 0).all())
    got = back.cpu().numpy().reshape(n, slot)
    assert np.array_equal(got[:, :fs], payload.reshape(n, fs))
    assert not got[:, fs:].any()          # the alignment padding is written as zeros


def test_plans_over_two_block_sum_steps():
    """4.3 M frames of 0-20 bytes: both plans have more than 16,384 blocks,
    so the block-sum scan takes two of its 16,384-sum steps, and the edge
    workgroups (67 K) are spread through the grid. Serialize and deserialize
    (align 1: every boundary mid-chunk) against the oracle."""
    n = 4_300_000
    rng = np.random.default_rng(43)
    payload = O.fill_splitmix(1 << 16, 43, 0)
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    sz = rng.integers(0, 21, n).astype(np.uint64)
    desc["payload_size"] = sz
    desc["payload_off"] = rng.integers(0, (1 << 16) - 32, n).astype(np.uint64)
    desc["fin"] = 1
    desc["opcode"] = 2
    desc["mask"] = (rng.random(n) < 0.7).astype(np.uint8)
    desc["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * desc["mask"]
    wire, total = check_serialize(payload, desc)
    offs, _ = W.wire_layout(desc)
    check_deserialize(wire[:total].copy(), offs, align=1)


def test_device_copy():
    """cfws_device_copy (the bench's copy ceiling) copies exactly, including
    sizes that end inside a wave's or a workgroup's span, and refuses
    misaligned arguments."""
    for n in (16, 1024, 2048 + 16, 4096 * 7 + 48, (8 << 20) + 16):
        src = torch.randint(0, 256, (n + 16,), dtype=torch.uint8, device="cuda")
        dst = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
        cfws.device_copy(src, dst, n)
        torch.cuda.synchronize()
        assert torch.equal(dst[:n], src[:n]) and int(dst[n:].sum()) == 0, n
    with pytest.raises(cfws.CodecError):
        cfws.device_copy(src, dst, 15)


def test_single_pass_plans_capacity_and_errors():
    """Plans of more than 2,048 blocks take the single-pass look-back form
    (one launch, no block-sum scan): 700 K frames of 0-40 bytes against the
    oracle, serialize cut by the capacity (the region map, the clamped
    total, the unclamped total reported), then deserialize the wire with
    invalid headers sprinkled in and a capacity that fails the later frames
    with OUT_OF_MEMORY; both the batch and the plan + execute calls."""
    n = 700_000
    rng = np.random.default_rng(71)
    payload = O.fill_splitmix(1 << 16, 71, 0)
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    desc["payload_size"] = rng.integers(0, 41, n).astype(np.uint64)
    desc["payload_off"] = rng.integers(0, (1 << 16) - 64, n).astype(np.uint64)
    desc["fin"] = 1
    desc["opcode"] = 2
    desc["mask"] = (rng.random(n) < 0.5).astype(np.uint8)
    desc["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * desc["mask"]
    wire, total = check_serialize(payload, desc)
    exp = wire[:total].copy()
    for pe in (False, True):
        cap = total // 2 + 3
        got, _, tot, _ = gpu_serialize(payload, desc, capacity=cap, plan_execute=pe)
        assert tot == total
        assert np.array_equal(got[:cap], exp[:cap]) and (got[cap:] == 0xEE).all()
    offs, _ = W.wire_layout(desc)
    bad = rng.choice(n, 300, replace=False)
    w = exp.copy()
    w[offs[bad].astype(np.int64)] |= 0x40                 # RSV2 -> INVALID_FRAME
    for pe in (False, True):
        check_deserialize(w, offs, align=1, plan_execute=pe)
        check_deserialize(w, offs, align=16, capacity=total // 3, plan_execute=pe)


def _mixed_desc(rng, n, payload_len, lo=80, hi=2000):
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    sz = rng.integers(lo, hi + 1, n).astype(np.uint64)
    desc["payload_size"] = sz
    desc["payload_off"] = (rng.integers(0, payload_len - 2048, n) & ~15).astype(np.uint64)
    desc["fin"] = (rng.random(n) < 0.8).astype(np.uint8)
    desc["opcode"] = rng.choice([0, 1, 2, 9], n).astype(np.uint8)
    desc["mask"] = (rng.random(n) < 0.7).astype(np.uint8)
    desc["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * desc["mask"]
    return desc


@pytest.mark.parametrize("n", [30_000, 600_000])
def test_serialize_in_region_edges(n):
    """WS serialize with in-region edge chunks (every payload 80..2,000 bytes,
    inside the 3,584-byte bound
    at a 16-aligned source offset: general_region_ser_edges writes each edge
    chunk with its segment): both plan forms (30 K frames: reduce + apply;
    600 K: the single-pass plan), masked and unmasked frames, 7- and 16-bit
    lengths, against the oracle; then a capacity cut inside the pass (the
    tail region's edge chunks stay with the edge workgroups), a batch whose
    total is a whole number of 4 KiB regions (no tail region), and the same
    frames with one 79-byte payload (the plan's flag off: edge workgroups
    write every edge chunk)."""
    rng = np.random.default_rng(n)
    payload = O.fill_splitmix(1 << 22, n, 0)
    desc = _mixed_desc(rng, n, 1 << 22)
    wire, total = check_serialize(payload, desc)
    exp = wire[:total].copy()
    for pe in (False, True):
        cap = total // 2 + 4101
        got, _, tot, _ = gpu_serialize(payload, desc, capacity=cap, plan_execute=pe)
        assert tot == total
        assert np.array_equal(got[:cap], exp[:cap]) and (got[cap:] == 0xEE).all()
    # total a multiple of the 4 KiB region: grow the last frames' payloads
    d2 = desc.copy()
    short = (-total) % 4096
    i = n - 1
    while short:
        add = min(short, 2000 - int(d2[i]["payload_size"]))
        if int(d2[i]["payload_size"]) <= 125 < int(d2[i]["payload_size"]) + add:
            add = 125 - int(d2[i]["payload_size"])          # keep the header size
        d2[i]["payload_size"] += add
        short -= add
        i -= 1
    _, t2 = W.wire_layout(d2)
    assert t2 % 4096 == 0
    check_serialize(payload, d2)
    d3 = desc.copy()
    d3[n // 2]["payload_size"] = 79
    check_serialize(payload, d3, plan_execute=True)


@pytest.mark.parametrize("case", ["mixed", "mixed3k", "half_regions", "mixed16k", "mixed64k", "region_starts",
                                  "64k"])
def test_serialize_aligned_large_frames(case):
    """WS serialize of payloads at 16-aligned source offsets past 2,000
    bytes -- the in-region send's bound (CFWS_SER_INREG_MAX) -- where a
    region holding a header is a one- or two-frame region: mixed 80 B-70 KB
    payloads, 1,800-3,584 bytes (in-region: one- and two-frame regions
    through general_region), 2,040-byte masked payloads (2,048 wire bytes:
    two frames per region, one starting on its boundary), and up to
    16,000 / 65,535 bytes (16-bit lengths: in-region under a raised
    CFWS_SER_INREG_MAX); 4,088-byte masked payloads (4,096 wire bytes:
    every frame starts on a region boundary); 64 KiB frames (14-byte
    headers: always the edge workgroups). Against
    the oracle, whole and cut at a capacity, through both launch forms."""
    rng = np.random.default_rng({"mixed": 1, "mixed3k": 6, "half_regions": 7, "mixed16k": 4, "mixed64k": 5,
                                 "region_starts": 2, "64k": 3}[case])
    payload = O.fill_splitmix(1 << 22, 77, 0)
    if case.startswith("mixed"):
        lo, hi = {"mixed": (80, 70000), "mixed3k": (1800, 3584), "mixed16k": (80, 16000),
                  "mixed64k": (80, 65535)}[case]
        desc = _mixed_desc(rng, 3000, 1 << 22, lo=lo, hi=hi)
        desc["payload_off"] = (rng.integers(0, (1 << 22) - hi - 16, 3000) & ~15).astype(np.uint64)
    elif case == "half_regions":
        desc = _mixed_desc(rng, 4000, 1 << 22)
        desc["payload_size"] = 2040                       # 2,048 wire bytes masked: two per region
        desc["mask"] = 1
        desc["mask_key"] = rng.integers(1, 1 << 32, 4000, dtype=np.uint64).astype(np.uint32)
    elif case == "region_starts":
        desc = _mixed_desc(rng, 2000, 1 << 22)
        desc["payload_size"] = 4088
        desc["mask"] = 1
        desc["mask_key"] = rng.integers(1, 1 << 32, 2000, dtype=np.uint64).astype(np.uint32)
        desc["payload_off"] = (rng.integers(0, (1 << 22) - 4096, 2000) & ~15).astype(np.uint64)
    else:
        desc = _mixed_desc(rng, 200, 1 << 22)
        desc["payload_size"] = 65536
        desc["payload_off"] = (rng.integers(0, (1 << 22) - 65536, 200) & ~15).astype(np.uint64)
    wire, total = check_serialize(payload, desc)
    if case == "region_starts":
        assert total == 4096 * 2000
    if case == "half_regions":
        assert total == 2048 * 4000
    exp = wire[:total].copy()
    for pe in (False, True):
        cap = total // 2 + 4101
        got, _, tot, _ = gpu_serialize(payload, desc, capacity=cap, plan_execute=pe)
        assert tot == total
        assert np.array_equal(got[:cap], exp[:cap]) and (got[cap:] == 0xEE).all()


@pytest.mark.parametrize("align", [16, 64, 4096])
def test_fused_deserialize_mixed_and_errors(align):
    """The fused deserialize (cfws_deserialize_batch on > 1,024 frames of
    <= 512 B average wire: deserialize_plan_single_kernel<true>, plan and
    copy in one pass) against the oracle and against plan + execute: frames
    of 0-40 bytes (64 frames per wave-instruction), 100-1,024 bytes, some
    of 1-9 KiB (frame by frame), masked and unmasked; invalid headers
    sprinkled in, a truncated last frame (MORE_DATA), a payload limit
    (TOO_BIG), and capacities that cut a slot and fail the frames past it
    with OUT_OF_MEMORY (their in-capacity slot bytes written as zeros)."""
    rng = np.random.default_rng(align)
    n = 120_000
    payload = O.fill_splitmix(1 << 16, align, 0)
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    kind = rng.random(n)
    sz = np.where(kind < 0.6, rng.integers(0, 41, n),
                  np.where(kind < 0.97, rng.integers(100, 1025, n), rng.integers(1025, 9000, n)))
    desc["payload_size"] = sz.astype(np.uint64)
    desc["payload_off"] = rng.integers(0, (1 << 16) - 9000, n).astype(np.uint64)
    desc["fin"] = 1
    desc["opcode"] = rng.choice([0, 1, 2, 9], n).astype(np.uint8)
    desc["mask"] = (rng.random(n) < 0.7).astype(np.uint8)
    desc["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * desc["mask"]
    exp_wire, d2 = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    offs = d2["wire_off"].astype(np.uint64)
    w = exp_wire.copy()
    bad = rng.choice(n - 1, 200, replace=False)
    w[offs[bad].astype(np.int64)] |= 0x40                      # RSV2 -> INVALID_FRAME
    w = w[:len(w) - 3]                                          # the last frame: MORE_DATA
    assert len(w) // n <= 512                                   # the fused form's batches
    out, d, st, tot = check_deserialize(w, offs, align=align)
    assert (st == O.ERROR_INVALID_FRAME).sum() >= 200 and st[-1] == O.PARSE_MORE_DATA
    ref = gpu_deserialize(w, offs, align=align, plan_execute=True)
    assert tot == ref[3] and np.array_equal(out[:tot], ref[0][:tot])
    check_deserialize(w, offs, align=align, max_payload=700)              # TOO_BIG
    for cap in (tot // 3 + 5, tot // 2):
        o2, _, s2, t2 = check_deserialize(w, offs, align=align, capacity=cap)
        assert (s2 == O.ERROR_OUT_OF_MEMORY).any() and t2 == cap
        r2 = gpu_deserialize(w, offs, align=align, capacity=cap, plan_execute=True)
        assert np.array_equal(o2[:cap], r2[0][:cap]) and (o2[cap:] == 0xEE).all()
