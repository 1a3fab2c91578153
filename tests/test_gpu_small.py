"""The single-launch small-batch path (serialize_small_kernel /
deserialize_small_kernel: <= 1,024 frames into <= 4 MiB) against the oracle
and against the plan + execute path on the same batch (a capacity above
4 MiB takes the latter): descriptors, statuses, totals and every output byte
the normal path writes, including headers across tiny frames, the capacity
cut, OUT_OF_MEMORY tails, alignment padding and MORE_DATA / invalid frames."""
import random

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402

BIG = (4 << 20) + 4096        # above the small path's capacity limit
PAYLOAD = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


def ser(payload_t, desc, cap, arena):
    d_t = cfws.desc_to_device(desc)
    wire = torch.full((arena,), 0xEE, dtype=torch.uint8, device="cuda")
    tot = cfws.serialize(payload_t, d_t, wire[:cap] if cap else wire[:0])
    torch.cuda.synchronize()
    return wire.cpu().numpy(), cfws.desc_from_device(d_t), int(tot.item())


@pytest.mark.parametrize("n,sizes", [(1, [0]), (1, [70000]), (7, [0, 1, 2, 3]),
                                     (256, [0, 1, 5, 13, 125, 126, 1000]),
                                     (1024, [0, 1, 2, 17, 125, 126, 127, 4000, 65535, 65536]),
                                     (1025, [1, 100])])
def test_small_serialize_equals_normal_and_oracle(n, sizes):
    rng = random.Random(n * 31 + len(sizes))
    payload = O.fill_splitmix(PAYLOAD, n, 0)
    pay_t = torch.from_numpy(payload).cuda()
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice(sizes)
        d[i] = (rng.randrange(0, PAYLOAD - sz), 0, sz, rng.getrandbits(32), rng.random() < .7,
                rng.choice([0, 1, 2, 8, 9, 10, 0x7f]), rng.random() < .6, 0)
    exp, exp_d = O.serialize_batch(payload, d.view(O.DESC_DTYPE))
    total = len(exp)
    arena = max(BIG, total + 16) + 64
    for cap in sorted({total, total + 5, (total + 15) // 16 * 16, max(total // 2, 1), BIG}):
        wire, got_d, tot = ser(pay_t, d, cap, arena)
        assert tot == total
        assert np.array_equal(got_d["wire_off"], exp_d["wire_off"])
        assert np.array_equal(got_d["header_size"], exp_d["header_size"])
        m = min(cap, total)
        assert np.array_equal(wire[:m], exp[:m]), cap
        if cap > total:
            # past the total: the last chunk's zeros within the capacity, then untouched
            end = min(cap, (total + 15) // 16 * 16)
            assert (wire[total:end] == 0).all() and (wire[end:cap] == 0xEE).all(), cap
        assert (wire[cap:] == 0xEE).all()


def test_small_serialize_matches_normal_bytes():
    """Same batch, small capacity (one launch) vs capacity > 4 MiB (plan +
    execute): identical wire arenas up to the capacity of the smaller."""
    rng = random.Random(77)
    payload = O.fill_splitmix(PAYLOAD, 77, 0)
    pay_t = torch.from_numpy(payload).cuda()
    n = 900
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 1, 3, 14, 15, 16, 17, 200, 3000])
        d[i] = (rng.randrange(0, PAYLOAD - sz), 0, sz, rng.getrandbits(32), 1, 2,
                rng.random() < .5, 0)
    small, d1, t1 = ser(pay_t, d, 1 << 20, BIG + 64)
    normal, d2, t2 = ser(pay_t, d, BIG, BIG + 64)
    assert t1 == t2
    assert np.array_equal(d1, d2)
    assert np.array_equal(small[:1 << 20], normal[:1 << 20])


def deser(wire_np, starts, cap, align, arena):
    wire_t = torch.from_numpy(np.concatenate([wire_np, np.zeros(32, np.uint8)])).cuda()
    idx = torch.from_numpy(np.asarray(starts, dtype=np.int64)).cuda()
    out = torch.full((arena,), 0xEE, dtype=torch.uint8, device="cuda")
    d, st, tot = cfws.deserialize(wire_t, len(wire_np), idx, out[:cap] if cap else out[:0], align=align)
    torch.cuda.synchronize()
    return out.cpu().numpy(), cfws.desc_from_device(d), st.cpu().numpy(), int(tot.item())


@pytest.mark.parametrize("n,align", [(1, 16), (5, 1), (300, 16), (700, 64), (1024, 1), (1030, 16)])
def test_small_deserialize_equals_oracle(n, align):
    rng = random.Random(n + align)
    frames = []
    for _ in range(n):
        p = rng.randbytes(rng.choice([0, 1, 2, 7, 15, 16, 17, 125, 126, 2000, 40000]))
        frames.append(O.serialize_keyed(rng.random() < .7, rng.choice([0, 1, 2, 9, 10, 3]),
                                        rng.random() < .6, rng.getrandbits(32), p))
    raw = bytearray(b"".join(frames))
    wire = np.frombuffer(bytes(raw), np.uint8).copy()
    starts, _ = O.index_frames(wire, n)
    starts = np.asarray(starts, dtype=np.uint64).copy()
    if n > 4:
        wire[int(starts[2])] = 0xF3                      # invalid opcode (-7001)
        starts[-1] = len(wire) - 1                       # MORE_DATA tail
    full = int(sum(((len(f) + align - 1) // align) * align for f in frames)) + 64
    arena = max(BIG, full) + 64
    for cap in sorted({full, full // 3, 0, BIG}):
        out, got_d, got_st, tot = deser(wire, starts, cap, align, arena)
        e_out, e_d, e_st, e_tot = O.deserialize_batch(wire, starts, align=align, capacity=cap)
        assert tot == e_tot, cap
        assert np.array_equal(got_st, e_st), cap
        for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask",
                  "header_size"):
            assert np.array_equal(got_d[f], e_d[f]), (cap, f)
        assert np.array_equal(out[:tot], e_out[:tot]), cap
        assert (out[cap:] == 0xEE).all()


@pytest.mark.parametrize("cap", [5_000_000, 5_000_003, 6_291_456 + 100])
def test_normal_path_capacity_cut_inside_a_body(cap):
    """Regression: a capacity above the small path's limit that cuts the pass
    inside a 64 KiB body. The streaming kernel's last region lay wholly in
    that body and was written to its end, past the caller's capacity; the
    pass-end region now clips every store at the capacity."""
    n, fs = 160, 65536
    payload = O.fill_splitmix(n * fs, 9, 0)
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * fs
    d["payload_size"], d["fin"], d["opcode"], d["mask"] = fs, 1, 2, 1
    d["mask_key"] = O.keys(9, n)
    exp, exp_d = O.serialize_batch(payload, d.view(O.DESC_DTYPE))
    arena = len(exp) + 8192
    wire, _, tot = ser(torch.from_numpy(payload).cuda(), d, cap, arena)
    assert tot == len(exp)
    assert np.array_equal(wire[:cap], exp[:cap]) and (wire[cap:] == 0xEE).all()
    # receive side: the same cut on the payload arena
    out, got_d, st, t = deser(exp, exp_d["wire_off"], cap, 16, arena)
    e_out, e_d, e_st, e_tot = O.deserialize_batch(exp, exp_d["wire_off"], align=16, capacity=cap)
    assert t == e_tot and np.array_equal(st, e_st)
    assert np.array_equal(out[:t], e_out[:t]) and (out[cap:] == 0xEE).all()
