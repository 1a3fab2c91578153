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
