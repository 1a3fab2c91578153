"""cfws_serialize_uniform (include/cfws.h): a batch of frames that share
payload size, fin, opcode and mask, serialized from a payload arena and one
4-byte key per frame, with no descriptor table and no plan.

The expectation is the oracle's sequential serialize of the same frames
(oracle serialize_batch, following co_ws_frame.c:21-119) -- which the
oracle's golden tests pin to the reference -- and the descriptor form
(cfws_serialize_batch) on the same device buffers, byte for byte over the
whole capacity. Full-size reference digests are in test_gpu_batch.py."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

SENT = 0xEE


def _frames(n, fs, mask, fin, opcode, seed):
    payload = O.fill_splitmix(max(n * fs, 16), 0x5EED0000 + seed, 0)[:n * fs]
    keys = O.keys(seed, n) if mask else np.zeros(n, np.uint32)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_off"] = np.arange(n, dtype=np.uint64) * np.uint64(fs)
    d["payload_size"], d["fin"], d["opcode"], d["mask"] = fs, fin, opcode, mask
    d["mask_key"] = keys
    return payload, keys, d


def _run(n, fs, mask=1, fin=1, opcode=2, seed=1, cap=None):
    payload, keys, d = _frames(n, fs, mask, fin, opcode, seed)
    exp, _ = O.serialize_batch(payload, d)
    total = len(exp)
    Wf = cfws.uniform_frame_bytes(fs, bool(mask))
    assert total == n * Wf
    cap = W.round16(total) + 32 if cap is None else cap
    pay_t = torch.from_numpy(np.concatenate([payload, np.zeros(16, np.uint8)])).cuda()
    keys_t = torch.from_numpy(keys.view(np.int32)).cuda() if mask else None
    wire = torch.full((max(cap, 1) + 64,), SENT, dtype=torch.uint8, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cfws.serialize_uniform(pay_t, keys_t, n, fs, wire, fin=bool(fin), opcode=opcode, mask=bool(mask),
                           total_t=tot, wire_capacity=cap)
    # the descriptor form on the same frames, into its own buffer
    wire2 = torch.full_like(wire, SENT)
    d_t = cfws.desc_to_device(d)
    ws = cfws.workspace(n, cap)
    tot2 = torch.zeros(1, dtype=torch.int64, device="cuda")
    if n:
        cfws._check(cfws.lib().cfws_serialize_batch(cfws._p(pay_t), cfws._p(d_t), n, cfws._p(wire2), cap,
                                                     cfws._p(tot2), cfws._p(ws), ws.numel(), cfws._stream(None)),
                    "cfws_serialize_batch")
    torch.cuda.synchronize()
    got = wire.cpu().numpy()
    assert int(tot.item()) == total
    lim = min(cap, total)
    bad = np.nonzero(got[:lim] != exp[:lim])[0]
    assert bad.size == 0, f"n={n} fs={fs} mask={mask}: {bad.size} bytes differ, first {bad[:8]}"
    # past the total, the last chunk writes zeros up to the capacity; nothing else is written
    z_end = min(cap, W.round16(total)) if total else 0
    assert (got[lim:max(lim, z_end)] == 0).all()
    assert (got[max(lim, z_end, cap):] == SENT).all()
    if n:
        assert torch.equal(wire, wire2), "differs from cfws_serialize_batch"
    return got


@pytest.mark.parametrize("fs", [0, 1, 2, 5, 9, 13, 14, 15, 16, 17, 100, 125, 126, 127, 240, 256, 257, 1000, 1023,
                                1024, 4096, 65535, 65536, 65537, 200_003])
@pytest.mark.parametrize("mask", [1, 0])
def test_uniform_sizes(fs, mask):
    """Payload sizes across the 7/16/64-bit length forms, frames shorter than
    a 16-byte chunk (the byte path), masked and not."""
    n = max(3, min(5000, (8 << 20) // max(fs + 14, 1)))
    _run(n, fs, mask)


@pytest.mark.parametrize("fin,opcode", [(1, 1), (0, 0), (1, 9), (1, 0x7F), (0, 0xFF)])
def test_uniform_header_bytes(fin, opcode):
    """b0 = opcode verbatim | 0x80 when fin (co_ws_frame.c:34-39)."""
    for fs in (7, 300, 70000):
        _run(64, fs, 1, fin, opcode, seed=fs)


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 1023, 4097])
def test_uniform_counts(n):
    for fs in (3, 250, 2000):
        _run(n, fs, 1, seed=n)


def test_uniform_capacity_cuts():
    """Wire bytes at or past the capacity are never written, at cuts inside
    headers, payloads and chunks."""
    for fs in (5, 256, 1000):
        total = 777 * cfws.uniform_frame_bytes(fs, True)
        for cap in (0, 1, 7, 16, 17, 33, total // 2 + 3, total - 17, total - 1, total):
            _run(777, fs, 1, cap=cap, seed=cap % 97)


def test_uniform_empty_and_arguments():
    wire = torch.full((64,), SENT, dtype=torch.uint8, device="cuda")
    tot = torch.full((1,), 5, dtype=torch.int64, device="cuda")
    pay = torch.zeros(64, dtype=torch.uint8, device="cuda")
    cfws.serialize_uniform(pay, None, 0, 100, wire, mask=False, total_t=tot)
    torch.cuda.synchronize()
    assert tot.item() == 0 and (wire == SENT).all()
    with pytest.raises(cfws.CodecError):                   # masked without keys
        cfws.serialize_uniform(pay, None, 2, 10, wire, mask=True)
    with pytest.raises(cfws.CodecError):                   # payload over 2^31
        cfws.serialize_uniform(pay, None, 1, (1 << 31) + 1, wire, mask=False)
    with pytest.raises(cfws.CodecError):                   # misaligned wire
        cfws.serialize_uniform(pay, None, 2, 10, wire[1:], mask=False)


# ---- the receive of a uniform stream (cfws_deserialize_slots_uniform) ------
# Frame i parsed at i * stride with no index: the expectation is the slot
# receive's (test_gpu_slots.expect_slots, the oracle's packed receive with the
# slot rule) over the index i * stride, the indexed info form on the same
# buffers, and the mismatch count of frames that are not COMPLETE frames of
# exactly `stride` bytes.

def _recv(wire, wire_size, n, stride, slot, cap=None, max_payload=O.DEFAULT_MAX_PAYLOAD, count=True):
    from test_gpu_slots import expect_slots
    cap = n * slot if cap is None else cap
    buf = np.full(W.round16(max(wire_size, 1)) + 32, SENT, np.uint8)
    buf[:wire_size] = wire[:wire_size]
    w = torch.from_numpy(buf).cuda()
    out = torch.full((W.round16(max(cap, 1)) + 32,), SENT, dtype=torch.uint8, device="cuda")
    out2 = torch.full_like(out, SENT)
    info = torch.full((max(n, 1), 8), SENT, dtype=torch.uint8, device="cuda")
    info2 = torch.full_like(info, SENT)
    mm = torch.full((1,), 12345, dtype=torch.int32, device="cuda") if count else None
    _, tot = cfws.deserialize_slots_uniform(w, wire_size, n, stride, out, slot, info, mismatch_t=mm,
                                            max_payload=max_payload, payload_capacity=cap)
    starts = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    if n:
        idx = torch.from_numpy(starts.view(np.int64)).cuda()
        _, tot2 = cfws.deserialize_slots_info(w, wire_size, idx, out2, slot, info2, max_payload=max_payload,
                                              payload_capacity=cap)
    torch.cuda.synchronize()
    e_arena, e_d, e_st, e_tot = expect_slots(wire, wire_size, starts, slot, cap, max_payload)
    assert int(tot.item()) == e_tot
    fi = info.cpu().numpy()[:n].reshape(-1).view(cfws.INFO_DTYPE)
    st = fi["status"].astype(np.int32)
    bad = np.nonzero(st != e_st)[0]
    assert bad.size == 0, f"{bad.size} statuses differ, first {[(int(i), int(st[i]), int(e_st[i])) for i in bad[:6]]}"
    assert np.array_equal(fi["payload_size"], np.minimum(e_d["payload_size"], np.uint64(0xFFFFFFFF)).astype(np.uint32))
    ok = e_st == O.PARSE_COMPLETE
    assert np.array_equal(fi["opcode"], e_d["opcode"]) and np.array_equal(fi["fin"][ok], e_d["fin"][ok])
    got = out.cpu().numpy()
    lim = W.round16(max(cap, 1))
    bad = np.nonzero(got[:lim] != e_arena)[0]
    assert bad.size == 0, f"{bad.size} arena bytes differ, first at {bad[:8]} (cap {cap})"
    assert (got[lim:] == SENT).all()
    if n:
        assert torch.equal(out, out2) and torch.equal(info, info2), "differs from the indexed info receive"
        assert int(tot2.item()) == e_tot
    odd = ~ok | (e_d["header_size"].astype(np.uint64) + e_d["payload_size"] != np.uint64(stride))
    if count:
        assert int(mm.item()) == int(odd.sum())
    return e_st, int(odd.sum())


@pytest.mark.parametrize("fs", [0, 1, 15, 16, 100, 125, 126, 240, 256, 512, 1000, 1024, 4064, 4096, 8160, 8161,
                                65535, 65536, 200_003])
@pytest.mark.parametrize("mask", [1, 0])
def test_uniform_receive_sizes(fs, mask):
    """The wire cfws_serialize_uniform writes, received with stride W into
    slots of round16(fs): every frame COMPLETE, no mismatch, the payload
    back; window kernels up to 8,160-byte slots, the per-frame kernel past."""
    n = max(3, min(4000, (6 << 20) // (fs + 14)))
    payload, keys, d = _frames(n, fs, mask, 1, 2, fs)
    wire, _ = O.serialize_batch(payload, d)
    stride = cfws.uniform_frame_bytes(fs, bool(mask))
    slot = max(16, W.round16(fs))
    st, odd = _recv(wire, len(wire), n, stride, slot)
    assert (st == O.PARSE_COMPLETE).all() and odd == 0


@pytest.mark.parametrize("stride", [2, 37, 262, 1000, 9001])
def test_uniform_receive_non_uniform_wire(stride):
    """A mixed batch (30-80 B frames, a 5,000-byte one every 97th) read at a
    fixed stride: frames land anywhere in headers and payloads -- invalid
    frames, MORE_DATA, OOM -- and the mismatch count says so."""
    from test_gpu_guard import _seed21_batch
    payload, desc = _seed21_batch(27)
    wire, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    n = min(len(desc), len(wire) // stride + 3)
    for slot in (96, 5008, 9008):                       # window kernels; pieces past 8,160 B
        _, odd = _recv(wire, len(wire), n, stride, slot)
        assert odd > 0
    _recv(wire, len(wire), n, stride, 96, max_payload=60)


def test_uniform_receive_truncated_and_cut():
    """The wire ends inside the last frames (MORE_DATA), slots too small for
    the payloads (OOM), capacities inside slots: each such frame counts."""
    n, fs = 3000, 256
    payload, keys, d = _frames(n, fs, 1, 1, 2, 9)
    wire, _ = O.serialize_batch(payload, d)
    stride = cfws.uniform_frame_bytes(fs, True)
    for cut, lost in ((len(wire) - 5, 1), (len(wire) - 3 * stride, 3), ((n - 10) * stride + 1, 10), (0, n)):
        st, odd = _recv(wire, cut, n, stride, 256)
        assert odd == lost and st[-1] == O.PARSE_MORE_DATA
    _, odd = _recv(wire, len(wire), n, stride, 240)
    assert odd == n
    for cap in (n * 256 // 2 + 5, n * 256 - 3, 17, 0):
        _, odd = _recv(wire, len(wire), n, stride, 256, cap=cap)
        assert odd == n - min(cap, n * 256) // 256
    for cut in (len(wire) - 5, (n - 10) * stride + 1):        # the piece kernel (slots over 8,160 B)
        _, odd = _recv(wire, cut, n, stride, 8192)
        assert odd == (1 if cut == len(wire) - 5 else 10)
    _recv(wire, len(wire), n, stride, 256, count=False)


def test_uniform_receive_arguments():
    w = torch.zeros(64, dtype=torch.uint8, device="cuda")
    out = torch.zeros(64, dtype=torch.uint8, device="cuda")
    info = torch.zeros((4, 8), dtype=torch.uint8, device="cuda")
    for stride in (0, 1):
        with pytest.raises(cfws.CodecError):
            cfws.deserialize_slots_uniform(w, 64, 4, stride, out, 16, info)
    with pytest.raises(cfws.CodecError):                   # n * stride past 2^63
        cfws.deserialize_slots_uniform(w, 64, 4, 1 << 62, out, 16, info)
    with pytest.raises(cfws.CodecError):                   # slot not a multiple of 16
        cfws.deserialize_slots_uniform(w, 64, 4, 20, out, 24, info)
    rc = cfws.lib().cfws_deserialize_slots_uniform(cfws._p(w), 64, 4, 20, 1 << 20, 16, None, cfws._p(out), 64,
                                                   None, None, cfws._stream(None))
    assert rc == cfws.ERROR_INVALID_ARGUMENT                # no info entries
    mm = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    tot = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    cfws.deserialize_slots_uniform(w, 64, 0, 20, out, 16, info, total_t=tot, mismatch_t=mm)
    torch.cuda.synchronize()
    assert mm.item() == 0 and tot.item() == 0


@pytest.mark.parametrize("fs,slot", [(4096, 16384), (3000, 65536), (2100, 8192), (9000, 20480), (1000, 16384),
                                     (256, 4096)])
def test_uniform_receive_slots_larger_than_frames(fs, slot):
    """Frames shorter than their slots: the piece kernel with fewer waves per
    frame than the slot has pieces (each wave taking every P-th piece), the
    window kernel, or the per-frame kernel, as the batch's average frame
    routes it -- against the oracle and the indexed receive."""
    n = 700
    payload, keys, d = _frames(n, fs, 1, 1, 2, fs + slot)
    wire, _ = O.serialize_batch(payload, d)
    stride = cfws.uniform_frame_bytes(fs, True)
    st, odd = _recv(wire, len(wire), n, stride, slot)
    assert (st == O.PARSE_COMPLETE).all() and odd == 0
