"""GPU bounds: every batch entry point over arenas that end (or start) at an
unmapped guard range, so one byte read or written outside an arena faults
at once (tests/native/guardmem.cpp: HIP virtual memory, the granules around
the arena reserved and never mapped).

Why ("The round-4 fault"): the first build of the fused
deserialize faulted with hipErrorIllegalAddress on every call that took it
(test_small_frame_regions_both_forms[21] and the 256 B / 1 KiB benches),
while the plan + execute digests of the same build passed. The suite's
arenas were padded (the wire with 16 spare bytes, the output with 16 per
frame), the bench's were exact 4 GiB-class allocations ending on a page
boundary. Here every arena is exact: the wire is total bytes (the library
reads whole aligned 16-byte blocks, so round16(total) is the readable end,
include/cfws.h), the output is the exact capacity, and writes between the
capacity and its 16-byte round-up are checked to leave the sentinel.
Every case is also compared with the oracle (bit-exact)."""
import ctypes as C
import os
import random

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
GUARD_LIB = os.path.join(HERE, "native", "libguardmem.so")


def _glib():
    if not hasattr(_glib, "L"):
        if not os.path.exists(GUARD_LIB):
            raise RuntimeError(f"{GUARD_LIB} missing: run `make` (it builds the guard helper)")
        L = C.CDLL(GUARD_LIB)
        L.guard_alloc.restype = C.c_uint64
        L.guard_alloc.argtypes = [C.c_uint64, C.c_int]
        L.guard_free.argtypes = [C.c_uint64]
        L.guard_copy.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.guard_fill.argtypes = [C.c_uint64, C.c_int, C.c_uint64]
        L.guard_last_error.restype = C.c_char_p
        _glib.L = L
    return _glib.L


class GuardBuf:
    """n bytes of device memory flush against an unmapped range: after its
    round16(n) end (flush_end) or before its start. Quacks like the 1-D
    uint8 tensors cfws.py takes (data_ptr, numel, shape, device)."""

    device = torch.device("cuda", 0)

    def __init__(self, n: int, flush_end: bool = True, fill: int | None = 0xEE):
        L = _glib()
        self.n = n
        self.ptr = L.guard_alloc(max(n, 1), 1 if flush_end else 0)
        assert self.ptr, L.guard_last_error().decode()
        if fill is not None:
            assert L.guard_fill(self.ptr, fill, W.round16(max(n, 1))) == 0
        self.flush_end = flush_end

    def data_ptr(self) -> int:
        return self.ptr

    def numel(self) -> int:
        return self.n

    @property
    def shape(self):
        return (self.n,)

    def upload(self, a: np.ndarray) -> "GuardBuf":
        a = np.ascontiguousarray(a, dtype=np.uint8)
        assert a.size <= W.round16(max(self.n, 1))
        torch.cuda.synchronize()
        if a.size:
            assert _glib().guard_copy(self.ptr, a.ctypes.data, a.size) == 0
        return self

    def download(self, n: int | None = None) -> np.ndarray:
        n = W.round16(max(self.n, 1)) if n is None else n
        out = np.empty(n, np.uint8)
        torch.cuda.synchronize()
        if n:
            assert _glib().guard_copy(out.ctypes.data, self.ptr, n) == 0, \
                _glib().guard_last_error().decode()
        return out

    def free(self) -> None:
        if self.ptr:
            assert _glib().guard_free(self.ptr) == 0, _glib().guard_last_error().decode()
            self.ptr = 0


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()
    torch.cuda.synchronize()
    if not _glib().guard_supported():
        pytest.skip("no HIP virtual memory management on this device")
    return torch.device("cuda", 0)


@pytest.fixture
def guards():
    bufs = []

    def make(n, flush_end=True, fill=0xEE):
        b = GuardBuf(n, flush_end, fill)
        bufs.append(b)
        return b
    yield make
    torch.cuda.synchronize()
    for b in bufs:
        b.free()


def _serialize(guards, payload, desc, flush_end, capacity=None, plan_execute=False):
    """cfws serialize into an exact wire arena; returns (wire bytes, total)."""
    pay = guards(max(payload.size, 16), flush_end).upload(payload)
    d_t = cfws.desc_to_device(desc)
    _, total = W.wire_layout(desc)
    cap = total if capacity is None else capacity
    wire = guards(max(cap, 1), flush_end)
    if plan_execute:
        ws = cfws.workspace(len(desc), cap)
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        cfws.serialize_plan(d_t, cap, tot, ws)
        cfws.serialize_execute(pay, d_t, wire, ws, cap)
    else:
        tot = cfws.serialize(pay, d_t, wire)
    torch.cuda.synchronize()
    assert int(tot.item()) == total
    got = wire.download()
    exp, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    c = min(cap, total)
    bad = np.nonzero(got[:c] != exp[:c])[0]
    assert bad.size == 0, f"{bad.size} wire bytes differ, first at {bad[:8]}"
    assert (got[max(cap, 1):] == 0xEE).all() if cap < W.round16(max(cap, 1)) else True, \
        "written past the wire capacity"
    return exp, total


def _deserialize(guards, wire, starts, flush_end, align=16, capacity=None, plan_execute=False,
                 wire_size=None):
    """cfws deserialize from an exact wire arena into an exact payload arena,
    against the oracle."""
    ws_n = len(wire) if wire_size is None else wire_size
    w = guards(max(ws_n, 1), flush_end).upload(wire[:ws_n])
    idx = torch.from_numpy(np.asarray(starts, dtype=np.int64)).cuda()
    e_out, e_d, e_st, e_tot = O.deserialize_batch(wire[:ws_n], starts, align=align,
                                                  capacity=capacity if capacity is not None else
                                                  len(wire) + 16 * len(starts) + 16)
    cap = capacity if capacity is not None else max(e_tot, 1)
    if capacity is None:      # exact: the oracle's total with the padded capacity is the need
        e_out, e_d, e_st, e_tot = O.deserialize_batch(wire[:ws_n], starts, align=align, capacity=cap)
    out = guards(cap, flush_end)
    n = len(starts)
    if plan_execute:
        wsp = cfws.workspace(n, cap)
        d_t = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        st_t = torch.empty(n, dtype=torch.int32, device="cuda")
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        cfws.deserialize_plan(w, ws_n, idx, d_t, st_t, cap, tot, wsp, align=align)
        cfws.deserialize_execute(w, d_t, st_t, out, wsp, cap)
    else:
        d_t, st_t, tot = cfws.deserialize(w, ws_n, idx, out, align=align)
    torch.cuda.synchronize()
    assert int(tot.item()) == e_tot
    assert np.array_equal(st_t.cpu().numpy(), e_st)
    d = cfws.desc_from_device(d_t)
    for f in ("payload_off", "payload_size", "mask_key", "opcode", "header_size"):
        assert np.array_equal(d[f], e_d[f]), f
    got = out.download()
    bad = np.nonzero(got[:e_tot] != e_out[:e_tot])[0]
    assert bad.size == 0, f"{bad.size} payload bytes differ, first at {bad[:8]}"
    assert (got[cap:] == 0xEE).all(), "written past the payload capacity"
    return e_st


def _seed21_batch(seed):
    """test_gpu_batch.test_small_frame_regions_both_forms's batch: 6,000
    frames of 30-80 B, a 5,000-byte frame every 97th (the round-4 fault's
    first failing case)."""
    rng = random.Random(seed)
    n = 6000
    payload = O.fill_splitmix(1 << 20, seed, 0)
    sizes = [rng.randrange(30, 80) for _ in range(n)]
    for i in range(0, n, 97):
        sizes[i] = 5000
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = sizes[i]
        desc[i] = (rng.randrange(0, (1 << 20) - sz), 0, sz, rng.getrandbits(32), rng.random() < .7,
                   rng.choice([0, 1, 2, 8, 9, 10]), rng.random() < .6, 0)
    return payload, desc


@pytest.mark.parametrize("flush_end", [True, False], ids=["end", "start"])
@pytest.mark.parametrize("seed", [21, 22])
def test_guard_small_mixed_both_forms(guards, seed, flush_end):
    payload, desc = _seed21_batch(seed)
    wire, total = _serialize(guards, payload, desc, flush_end)
    starts, consumed = O.index_frames(wire, len(desc) + 1)
    assert consumed == total
    for align in (1, 16):
        _deserialize(guards, wire, starts, flush_end, align=align)                 # fused at 16
        _deserialize(guards, wire, starts, flush_end, align=align, plan_execute=True)


@pytest.mark.parametrize("fs", [0, 1, 125, 126, 256, 1024, 2048, 3072, 3584, 4096, 65536])
def test_guard_uniform_sizes(guards, fs):
    """Uniform batches (the bench's shape at ~32 MiB): the single-pass plans
    above 524,288 frames are covered by the full-size case below."""
    n = max(64, min(200_000, (32 << 20) // max(fs, 1)))
    desc = W.uniform_batch(n, fs, 2, opcode=cfws.OPCODE_BINARY)
    payload = O.fill_splitmix(max(n * fs, 16), 0x5EED0002, 0)[:n * fs]
    wire, total = _serialize(guards, payload, desc, True)
    _serialize(guards, payload, desc, True, plan_execute=True)
    offs, _ = W.wire_layout(desc)
    _deserialize(guards, wire, offs, True)
    _deserialize(guards, wire, offs, True, plan_execute=True)


def test_guard_capacity_cuts(guards):
    """Capacities that end inside a frame, at odd byte counts: every store
    must stop at the capacity (fused store tail, tail_region)."""
    payload, desc = _seed21_batch(23)
    wire, total = _serialize(guards, payload, desc, True)
    for cap in (total // 2 + 5, total - 3, 4097):
        _serialize(guards, payload, desc, True, capacity=cap)
    starts, _ = O.index_frames(wire, len(desc) + 1)
    full = O.deserialize_batch(wire, starts, align=16, capacity=len(wire) + 16 * len(starts))[3]
    for cap in (full // 2 + 7, full - 1, 1001):
        _deserialize(guards, wire, starts, True, align=16, capacity=cap)
        _deserialize(guards, wire, starts, True, align=1, capacity=cap, plan_execute=True)


def test_guard_truncated_wire(guards):
    """The wire ends inside the last frame (MORE_DATA) at every offset of
    its header and into its payload: the header loads near the arena end."""
    payload, desc = _seed21_batch(24)
    desc = desc[:2000]
    wire, total = _serialize(guards, payload, desc, True)
    starts, _ = O.index_frames(wire, len(desc) + 1)
    last = int(starts[-1])
    for cut in (last + 1, last + 2, last + 3, last + 7, total - 1):
        st = _deserialize(guards, wire, starts, True, wire_size=cut)
        assert st[-1] == O.PARSE_MORE_DATA


def test_guard_split_ops(guards):
    """encode_headers + mask_batch (both forms) into an exact wire, then
    parse_headers + unmask_batch from it into an exact, packed payload arena."""
    payload, desc = _seed21_batch(25)
    exp_wire, d_exp = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    total = len(exp_wire)
    d = desc.copy()
    d["wire_off"] = d_exp["wire_off"]
    mp = int(d["payload_size"].max())
    pay = guards(payload.size).upload(payload)
    for packed in (False, True):
        wire = guards(total)
        d_t = cfws.desc_to_device(d)
        cfws.encode_headers(d_t, wire)
        cfws.mask_batch(pay, d_t, wire, mp, packed=packed)
        torch.cuda.synchronize()
        got = wire.download()
        assert np.array_equal(got[:total], exp_wire), packed
        assert (got[total:] == 0xEE).all()
    idx = torch.from_numpy(d_exp["wire_off"].astype(np.int64)).cuda()
    pd = torch.empty((len(d), 32), dtype=torch.uint8, device="cuda")
    ps = torch.empty(len(d), dtype=torch.int32, device="cuda")
    cfws.parse_headers(wire, total, idx, pd, ps)
    torch.cuda.synchronize()
    e_d, e_st = O.parse_headers(exp_wire, d_exp["wire_off"])
    got_d = cfws.desc_from_device(pd)
    assert np.array_equal(ps.cpu().numpy(), e_st) and (e_st == 0).all()
    for f in ("payload_size", "mask_key", "mask", "header_size"):
        assert np.array_equal(got_d[f], e_d[f]), f
    sizes = got_d["payload_size"].astype(np.uint64)
    got_d["payload_off"] = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    e_d["payload_off"] = got_d["payload_off"]
    n_out = int(sizes.sum())
    back = guards(n_out)
    cfws.unmask_batch(wire, cfws.desc_to_device(got_d), ps, back, mp)
    exp_back = np.zeros(n_out, np.uint8)
    O.unmask_batch(exp_wire, e_d, e_st, exp_back)
    torch.cuda.synchronize()
    got = back.download()
    assert np.array_equal(got[:n_out], exp_back)
    assert (got[n_out:] == 0xEE).all()


def test_guard_h2_roundtrip(guards):
    rng = random.Random(5)
    payload = O.fill_splitmix(1 << 21, 5, 0)
    n = 3000
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 1, 125, 126, 999, 16376, 16377, 40000])
        d[i] = (rng.randrange(0, (1 << 21) - sz), 0, sz, rng.getrandbits(32), True,
                rng.choice([1, 2]), rng.random() < .8, 0)
    exp, _ = O.h2_serialize_batch(payload, d, 3, 16384)
    pay = guards(payload.size).upload(payload)
    _, wtotal = W.wire_layout(d)
    wire = guards(wtotal)
    h2 = guards(len(exp))
    tot = cfws.h2_serialize(pay, cfws.desc_to_device(d), wire, h2, 3, 16384)
    torch.cuda.synchronize()
    assert int(tot.item()) == len(exp)
    assert np.array_equal(h2.download(len(exp)), exp)
    index = O.h2_index(exp)
    e = O.h2_deserialize_batch(exp, index, 16384)
    pool = guards(len(exp))
    out = guards(max(e["total"], 1))
    idx = torch.from_numpy(index.astype(np.int64)).cuda()
    st, md, ms, t, m = cfws.h2_deserialize(h2, len(exp), idx, pool, out)
    torch.cuda.synchronize()
    assert m == e["n_msg"] and int(t.item()) == e["total"]
    assert np.array_equal(ms.cpu().numpy(), e["msg_status"])
    got = out.download()
    assert np.array_equal(got[:e["total"]], e["payload"][:e["total"]])
    assert (got[max(e["total"], 1):] == 0xEE).all()


def test_guard_index_frames(guards):
    payload, desc = _seed21_batch(26)
    wire, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    total = len(wire)
    buf = guards(total).upload(wire)
    cuts = [0, 1000, 50_000, 120_000, total]
    begin = torch.tensor(cuts[:-1], dtype=torch.int64, device="cuda")
    end = torch.tensor(cuts[1:], dtype=torch.int64, device="cuda")
    starts, first, consumed, stop, k = cfws.index_frames_batch(buf, begin, end)
    torch.cuda.synchronize()
    for c in range(len(cuts) - 1):
        es, ec, estop = O.index_stream(wire, cuts[c], cuts[c + 1])
        assert int(consumed[c]) == ec and int(stop[c]) == estop


@pytest.mark.parametrize("fs", [256, 1024])
def test_guard_bench_shape_full_size(guards, fs):
    """The benches that faulted in round 4 (16 M x 256 B, 4 M x 1 KiB; 4 GiB of
    payload), with exact arenas: payload, wire and unmasked copy each end at
    an unmapped range. Serialize plan + execute, the one-call deserialize
    (the fused kernel at 256 B), and the round trip compared on the device."""
    n = (4 << 30) // fs
    desc = W.uniform_batch(n, fs, 2, opcode=cfws.OPCODE_BINARY)
    offs, total = W.wire_layout(desc)
    pay = guards(n * fs, fill=None)
    cfws.fill_splitmix(pay, 0x5EED0002)
    d_t = cfws.desc_to_device(desc)
    wire = guards(total, fill=None)
    tot = cfws.serialize(pay, d_t, wire)
    torch.cuda.synchronize()
    assert int(tot.item()) == total
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    back = guards(n * fs, fill=None)
    _, st, ptot = cfws.deserialize(wire, total, idx, back, align=16)
    torch.cuda.synchronize()
    assert int(ptot.item()) == n * fs and bool((st == 0).all())
    # compare on the device, 256 MiB at a time
    a = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    L = _glib()
    for o in range(0, n * fs, a.numel()):
        k = min(a.numel(), n * fs - o)
        assert L.guard_copy(a.data_ptr(), pay.ptr + o, k) == 0
        assert L.guard_copy(b.data_ptr(), back.ptr + o, k) == 0
        assert torch.equal(a[:k], b[:k]), o
