"""cfws_deserialize_slots (include/cfws.h): frame i's payload at i * slot.

The expectation is the oracle's own parse and unmask (oracle
deserialize_batch, following co_ws_frame.c:121-247) relocated into slot i:
the slot layout is this library's (the slab form of the reference's one
allocation per frame, co_ws_frame.c:216-223), so the relocation and the slot
rule are restated here, in the test. Every arena is guarded
(tests/native/guardmem.cpp): the wire ends at its round16(wire_size), the
payload arena at round16(capacity), and bytes past the capacity, past each
payload's 16-byte round-up and in the slots of non-COMPLETE frames are
checked to keep their sentinel. Slots up to 992 bytes take the window
kernel with one block per lane, up to 2,016 with two, up to 4,064 with
four, up to 8,160 with eight, larger ones the per-frame kernel.

Every case runs in both output forms (the `form` fixture): descriptors +
statuses (cfws_deserialize_slots / _scatter) and the compact 8-byte
cfws_frame_info_t (cfws_deserialize_slots_info / _scatter_info, in a guarded
buffer of exactly 8 n bytes)."""
import random

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402
from test_gpu_guard import GuardBuf, _glib, _seed21_batch  # noqa: E402

SENT = 0xEE


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()
    torch.cuda.synchronize()
    if not _glib().guard_supported():
        pytest.skip("no HIP virtual memory management on this device")
    return torch.device("cuda", 0)


FORM = {"form": "desc"}


@pytest.fixture(params=["desc", "info"], autouse=True)
def form(request):
    FORM["form"] = request.param
    yield request.param
    FORM["form"] = "desc"


@pytest.fixture
def guards():
    bufs = []

    def make(n, flush_end=True):
        b = GuardBuf(n, flush_end, SENT)
        bufs.append(b)
        return b
    yield make
    torch.cuda.synchronize()
    for b in bufs:
        b.free()


def expect_slots(wire, wire_size, starts, slot, cap, max_payload=O.DEFAULT_MAX_PAYLOAD, offs=None):
    """(arena of round16(cap) bytes, desc, status, total) as
    cfws_deserialize_slots defines them, from the oracle's packed receive;
    with offs, as cfws_deserialize_scatter does (frame i at offs[i], which
    must be a multiple of 16; slot is then max_slot; total is None)."""
    n = len(starts)
    # packed with room for every COMPLETE payload (indices may repeat)
    p_d, p_st = O.parse_headers(wire[:wire_size], starts, max_payload)
    room = int(p_d["payload_size"][p_st == O.PARSE_COMPLETE].sum()) + 16
    e_out, e_d, e_st, _ = O.deserialize_batch(wire[:wire_size], starts, align=1, max_payload=max_payload,
                                              capacity=room)
    ps = e_d["payload_size"].astype(np.uint64)
    run = np.arange(n, dtype=np.uint64) * np.uint64(slot) if offs is None else np.asarray(offs, np.uint64)
    st = e_st.copy()
    fits = (ps <= slot) & (run <= np.uint64(cap)) & (ps <= np.uint64(cap) - np.minimum(run, np.uint64(cap)))
    if offs is not None:
        fits &= (run % np.uint64(16)) == 0
    oom = (st == O.PARSE_COMPLETE) & (ps > 0) & ~fits
    st[oom] = O.ERROR_OUT_OF_MEMORY
    arena = np.full(W.round16(max(cap, 1)), SENT, np.uint8)
    for i in np.nonzero((st == O.PARSE_COMPLETE) & (ps > 0))[0]:
        r, L, o = int(run[i]), int(ps[i]), int(e_d["payload_off"][i])
        arena[r:r + L] = e_out[o:o + L]
        arena[r + L:min(r + W.round16(L), cap)] = 0
    d = e_d.copy()
    d["payload_off"] = run
    return arena, d, st, (min(n * slot, cap) if offs is None else None)


def run_slots(guards, wire, starts, slot, cap=None, wire_size=None, max_payload=O.DEFAULT_MAX_PAYLOAD,
              flush_end=True, offs=None):
    """cfws_deserialize_slots, or with offs cfws_deserialize_scatter (slot
    is then max_slot), against expect_slots."""
    ws_n = len(wire) if wire_size is None else wire_size
    n = len(starts)
    cap = n * slot if cap is None else cap
    w = guards(max(ws_n, 1), flush_end).upload(wire[:ws_n])
    out = guards(max(cap, 1), flush_end)
    idx = torch.from_numpy(np.asarray(starts, dtype=np.uint64).view(np.int64)).cuda()
    info = FORM["form"] == "info"
    inf_b = guards(max(8 * n, 1), flush_end) if info else None
    off_t = None if offs is None else torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).cuda()
    tot = None
    if offs is None and info:
        _, tot = cfws.deserialize_slots_info(w, ws_n, idx, out, slot, inf_b, max_payload=max_payload,
                                             payload_capacity=cap)
    elif offs is None:
        d_t, st_t, tot = cfws.deserialize_slots(w, ws_n, idx, out, slot, max_payload=max_payload,
                                                payload_capacity=cap)
    elif info:
        cfws.deserialize_scatter_info(w, ws_n, idx, off_t, out, slot, inf_b, max_payload=max_payload,
                                      payload_capacity=cap)
    else:
        d_t, st_t = cfws.deserialize_scatter(w, ws_n, idx, off_t, out, slot, max_payload=max_payload,
                                             payload_capacity=cap)
    torch.cuda.synchronize()
    e_arena, e_d, e_st, e_tot = expect_slots(wire, ws_n, starts, slot, cap, max_payload, offs)
    if tot is not None:
        assert int(tot.item()) == e_tot
    ok = e_st == O.PARSE_COMPLETE
    if info:
        fi = inf_b.download()[:8 * n].view(cfws.INFO_DTYPE)
        st = fi["status"].astype(np.int32)
        bad = np.nonzero(st != e_st)[0]
        assert bad.size == 0, f"{bad.size} statuses differ, first {[(int(i), int(st[i]), int(e_st[i])) for i in bad[:6]]}"
        e_ps = np.minimum(e_d["payload_size"], np.uint64(0xFFFFFFFF)).astype(np.uint32)
        assert np.array_equal(fi["payload_size"], e_ps), "payload_size"
        assert np.array_equal(fi["opcode"], e_d["opcode"]), "opcode"
        assert np.array_equal(fi["fin"][ok], e_d["fin"][ok]), "fin"
    else:
        st = st_t.cpu().numpy()
        bad = np.nonzero(st != e_st)[0]
        assert bad.size == 0, f"{bad.size} statuses differ, first {[(int(i), int(st[i]), int(e_st[i])) for i in bad[:6]]}"
        d = cfws.desc_from_device(d_t)
        for f in ("payload_off", "wire_off", "payload_size", "mask_key", "opcode", "header_size"):
            assert np.array_equal(d[f], e_d[f]), f
        for f in ("fin", "mask"):
            assert np.array_equal(d[f][ok], e_d[f][ok]), f
    got = out.download()
    bad = np.nonzero(got != e_arena)[0]
    assert bad.size == 0, f"{bad.size} arena bytes differ, first at {bad[:8]} (cap {cap})"
    return e_st


def _wire_of(payload, desc):
    wire, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    starts, consumed = O.index_frames(wire, len(desc) + 1)
    assert consumed == len(wire)
    return wire, starts


@pytest.mark.parametrize("slot", [16, 48, 80, 256, 512, 992, 1008, 1504, 2016, 2032, 3008, 4064, 4080, 6000, 8160, 8176])
@pytest.mark.parametrize("seed", [21, 22])
def test_slots_mixed(guards, seed, slot):
    """6,000 frames of 30-80 B (masked and not, data and control) with a
    5,000-byte frame every 97th: at slots under 80 B some frames are OOM,
    under 5,000 B the long ones are."""
    payload, desc = _seed21_batch(seed)
    wire, starts = _wire_of(payload, desc)
    st = run_slots(guards, wire, starts, slot)
    if slot >= 80:
        assert (st == O.PARSE_COMPLETE).any()
    if slot < 5000:
        assert (st == O.ERROR_OUT_OF_MEMORY).any()


@pytest.mark.parametrize("flush_end", [True, False], ids=["end", "start"])
@pytest.mark.parametrize("slot", [256, 1504, 3008, 4096, 8208])
def test_slots_guard_start(guards, slot, flush_end):
    payload, desc = _seed21_batch(25)
    wire, starts = _wire_of(payload, desc)
    run_slots(guards, wire, starts, slot, flush_end=flush_end)


@pytest.mark.parametrize("fs", [0, 1, 125, 126, 240, 256, 977, 992, 1000, 1024, 2000, 2016, 2017, 3072, 4064, 4065, 8160, 8161, 65536])
def test_slots_uniform(guards, fs):
    """Uniform batches at slot = round16(fs) (at least 16): the bench's shape,
    every frame COMPLETE and every slot full."""
    n = max(64, min(150_000, (24 << 20) // max(fs, 1)))
    desc = W.uniform_batch(n, fs, 2, opcode=cfws.OPCODE_BINARY)
    payload = O.fill_splitmix(max(n * fs, 16), 0x5EED0003, 0)[:n * fs]
    wire, starts = _wire_of(payload, desc)
    st = run_slots(guards, wire, starts, max(16, W.round16(fs)))
    assert (st == O.PARSE_COMPLETE).all()


def test_slots_capacity_cuts(guards):
    """Capacities inside a slot and inside a payload, at odd byte counts."""
    payload, desc = _seed21_batch(23)
    wire, starts = _wire_of(payload, desc)
    n = len(starts)
    for slot in (96, 1504, 6016):
        for cap in (n * slot // 2 + 5, n * slot - 3, 1001, 17, 0):
            run_slots(guards, wire, starts, slot, cap=cap)


def test_slots_truncated_wire(guards):
    """The wire ends inside the last frame, at every offset of its header
    and into its payload (MORE_DATA), and starts past the wire's end."""
    payload, desc = _seed21_batch(24)
    desc = desc[:2000]
    wire, starts = _wire_of(payload, desc)
    last = int(starts[-1])
    for slot in (128, 1504, 5008):
        for cut in (last + 1, last + 2, last + 3, last + 7, len(wire) - 1):
            st = run_slots(guards, wire, starts, slot, wire_size=cut)
            assert st[-1] == O.PARSE_MORE_DATA


def test_slots_any_index(guards):
    """Indices in any order, repeated, inside payloads (whatever header the
    bytes there make: invalid frames, DATA_TOO_BIG, MORE_DATA) and past the
    wire's end; a small max_payload."""
    payload, desc = _seed21_batch(26)
    wire, starts = _wire_of(payload, desc)
    rng = random.Random(26)
    idx = list(starts)
    idx += [rng.randrange(0, len(wire)) for _ in range(3000)]
    idx += [len(wire), len(wire) + 5, (1 << 40), (1 << 64) - 1]
    idx += list(starts[:500])
    rng.shuffle(idx)
    idx = np.array(idx, dtype=np.uint64)
    for slot in (64, 256, 992, 1504, 2048, 4080, 8192):
        st = run_slots(guards, wire, idx, slot)
        assert (st == O.ERROR_INVALID_FRAME).any() and (st == O.PARSE_MORE_DATA).any()
        run_slots(guards, wire, idx, slot, max_payload=60)


def test_slots_arguments(guards):
    wire = np.zeros(64, np.uint8)
    w = guards(64).upload(wire)
    out = guards(64)
    idx = torch.zeros(1, dtype=torch.int64, device="cuda")
    for slot in (0, 8, 24, (1 << 31) + 16):
        with pytest.raises(cfws.CodecError):
            cfws.deserialize_slots(w, 64, idx, out, slot)
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    _, _, tot = cfws.deserialize_slots(w, 64, e, out, 16, total_t=torch.full((1,), 7, dtype=torch.int64,
                                                                                device="cuda"))
    torch.cuda.synchronize()
    assert tot.item() == 0


@pytest.mark.parametrize("slot", [16, 256, 2048, 16384])
def test_slots_tiny_wires(guards, slot):
    """Wires of 0 to 40 bytes (the header parsed from single bytes below 16,
    window blocks cut at the wire's end), one to three frames."""
    frames = [(bytes(range(3)), 0x0A0B0C0D), (b"", None), (bytes(range(9)), None)]
    sizes = np.array([len(p) for p, _ in frames], dtype=np.uint64)
    desc = np.zeros(3, dtype=O.DESC_DTYPE)
    desc["payload_size"] = sizes
    desc["payload_off"] = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64)
    desc["fin"], desc["opcode"] = 1, 1
    desc["mask"] = [1, 0, 0]
    desc["mask_key"] = [0x0A0B0C0D, 0, 0]
    arena = np.frombuffer(b"".join(p for p, _ in frames), np.uint8).copy()
    wire, _ = O.serialize_batch(arena, desc)
    starts, _ = O.index_frames(wire, 4)
    for cut in range(0, len(wire) + 1, 3):
        run_slots(guards, wire, starts, slot, wire_size=cut)


def _scatter_offsets(n, max_slot, rng, cap_slack=0):
    """Non-overlapping 16-aligned destinations in a shuffled order with gaps
    of 0-48 bytes: frame i's region is [offs[i], offs[i] + max_slot)."""
    stride = max_slot + 64
    perm = rng.permutation(n).astype(np.uint64)
    return perm * np.uint64(stride) + rng.integers(0, 4, n).astype(np.uint64) * np.uint64(16), n * stride + cap_slack


@pytest.mark.parametrize("max_slot", [16, 96, 256, 1504, 4064, 8160, 16384])
def test_scatter_permuted(guards, max_slot):
    """cfws_deserialize_scatter over every kernel (window with one to eight
    blocks per lane, per-frame): destinations shuffled, with gaps left
    untouched, and frames too long for max_slot OUT_OF_MEMORY."""
    payload, desc = _seed21_batch(31)
    wire, starts = _wire_of(payload, desc)
    rng = np.random.default_rng(max_slot)
    offs, cap = _scatter_offsets(len(starts), max_slot, rng)
    run_slots(guards, wire, starts, max_slot, cap=cap, offs=offs)


@pytest.mark.parametrize("fs,max_slot", [(9000, 9008), (4096, 4096), (2048, 2048), (20000, 20480), (3000, 16384)])
def test_scatter_pieces(guards, fs, max_slot):
    """The piece kernel through the scatter form (frames that fill their
    slots, or average past 1 KiB in slots over 8,160 B): shuffled
    destinations with gaps, and a capacity that cuts the last slots."""
    n = max(40, min(600, (6 << 20) // max_slot))
    desc = W.uniform_batch(n, fs, 5, opcode=cfws.OPCODE_BINARY)
    payload = O.fill_splitmix(n * fs, 0x5EED0005, 0)
    wire, starts = _wire_of(payload, desc)
    assert cfws.lib().cfws_deserialize_slots_pass_kernel(n, len(wire), max_slot).decode() == \
        "deserialize_slots_piece_kernel"
    rng = np.random.default_rng(fs)
    offs, cap = _scatter_offsets(n, max_slot, rng)
    run_slots(guards, wire, starts, max_slot, cap=cap, offs=offs)
    run_slots(guards, wire, starts, max_slot, cap=cap - 3 * max_slot - 5, offs=offs)


def test_scatter_bad_offsets(guards):
    """Offsets that are not multiples of 16, that end past the capacity, or
    that are near 2^64 (no wrap): OUT_OF_MEMORY, nothing written for them."""
    payload, desc = _seed21_batch(32)
    wire, starts = _wire_of(payload, desc)
    n = len(starts)
    rng = np.random.default_rng(32)
    offs, cap = _scatter_offsets(n, 5008, rng)
    offs = offs.copy()
    offs[::7] += np.uint64(8)                       # misaligned
    offs[3::11] = np.uint64(cap - 16)              # ends past the capacity (unless tiny)
    offs[5::13] = np.uint64((1 << 64) - 16)         # would wrap
    for max_slot in (256, 5008):
        st = run_slots(guards, wire, starts, max_slot, cap=cap, offs=offs)
        assert (st == O.ERROR_OUT_OF_MEMORY).any() and (st == O.PARSE_COMPLETE).any()
