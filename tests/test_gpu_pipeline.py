"""GPU parity of the host-memory pipeline (cfws_pipeline_*): host buffers in,
host buffers out, H2D / kernels / D2H overlapped over several slots; results
must equal the oracle's (which is pinned to the reference) byte for byte,
however the batch is cut into chunks."""
import random

import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402


HOST = {"kind": "torch", "d2h": None}


def pinned(n: int):
    """Host buffer of the kind under test: torch's pinned memory (the
    pipeline's D2H leg is an SDMA copy) or mapped pinned memory (the D2H leg
    is copy_out_kernel writing it over PCIe)."""
    if HOST["kind"] == "mapped":
        t = cfws.mapped_host(n)
        t.zero_()
    else:
        t = torch.zeros(max(n, 16), dtype=torch.uint8, pin_memory=True)
    return t, t.numpy()


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


@pytest.fixture(autouse=True, params=["torch", "mapped", "mapped-kernel", "mapped-dma"])
def host_kind(request):
    """Host arenas x the pipeline's D2H mode: torch pinned memory (SDMA
    whatever the mode), mapped memory with the default mode (serialize by
    kernel, deserialize by SDMA) and with each direction forced."""
    kind, _, d2h = request.param.partition("-")
    HOST["kind"], HOST["d2h"] = kind, d2h or None
    yield kind
    HOST["kind"], HOST["d2h"] = "torch", None


def make_pipeline(**kw):
    return cfws.Pipeline(d2h=HOST["d2h"], **kw)


def test_copy_to_host_any_alignment():
    src = torch.from_numpy(O.fill_splitmix(1 << 20, 5)).cuda()
    out_t, out = pinned((1 << 20) + 64)
    if HOST["kind"] == "torch":
        # not mapped memory: refused, nothing written
        with pytest.raises(cfws.CodecError):
            cfws.copy_to_host(src, out_t.data_ptr(), 100)
        return
    exp = out.copy()
    for so, do, n in [(0, 0, 1 << 20), (3, 5, 1000), (16, 1, 17), (7, 7, 65536 + 9), (1, 0, 15),
                      (0, 33, 0)]:
        cfws.copy_to_host(src[so:], out_t.data_ptr() + do, n)
        torch.cuda.synchronize()
        exp[do:do + n] = src[so:so + n].cpu().numpy()
        assert np.array_equal(out, exp), (so, do, n)


@pytest.mark.parametrize("chunk,depth", [(69632, 1), (69632, 3), (1 << 20, 2)])
def test_pipeline_serialize_matches_oracle(chunk, depth):
    rng = random.Random(chunk + depth)
    payload_t, payload = pinned(3 << 20)
    payload[:] = O.fill_splitmix(payload.size, 77, 0)
    n = 3000
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    off = 0
    for i in range(n):
        sz = rng.choice([0, 1, 5, 125, 126, 1000, 4000, 20000, 65535, 65536, 65537 - 40000])
        if rng.random() < 0.5:
            off = rng.randrange(0, payload.size - sz)       # jump around
        d[i] = (off, 0, sz, rng.getrandbits(32), rng.random() < .7, rng.choice([0, 1, 2, 9]),
                rng.random() < .6, 0)
        off = min(off + sz, payload.size - 70000)
    exp, exp_d = O.serialize_batch(payload, d.view(O.DESC_DTYPE))
    wire_t, wire = pinned(len(exp) + 64)
    p = make_pipeline(chunk_bytes=chunk, max_frames=512, depth=depth)
    tot = p.serialize(payload_t.data_ptr(), d, wire_t.data_ptr(), wire.size)
    p.close()
    assert tot == len(exp)
    assert np.array_equal(d["wire_off"], exp_d["wire_off"])
    assert np.array_equal(wire[:tot], exp)


@pytest.mark.parametrize("chunk,depth,align", [(69632, 1, 16), (69632, 3, 1), (1 << 20, 2, 64)])
def test_pipeline_deserialize_matches_oracle(chunk, depth, align):
    rng = random.Random(chunk + depth + align)
    frames = []
    for _ in range(2500):
        p = rng.randbytes(rng.choice([0, 1, 7, 125, 126, 3000, 20000, 40000]))
        frames.append(O.serialize_keyed(rng.random() < .7, rng.randrange(16), rng.random() < .6,
                                        rng.getrandbits(32), p))
    raw = b"".join(frames)
    wire_t, wire = pinned(len(raw))
    wire[:len(raw)] = np.frombuffer(raw, np.uint8)
    starts, _ = O.index_frames(wire[:len(raw)], 100000)
    starts = np.concatenate([starts, [len(raw) - 1, len(raw)]]).astype(np.uint64)  # truncated tails
    pl = make_pipeline(chunk_bytes=chunk, max_frames=300, depth=depth)
    for cap in (len(raw) + align * len(starts) + 64, len(raw) // 2):
        out_t, out = pinned(cap)
        desc, st, tot = pl.deserialize(wire_t.data_ptr(), len(raw), starts, out_t.data_ptr(), cap,
                                       align=align)
        e_out, e_d, e_st, e_tot = O.deserialize_batch(wire[:len(raw)], starts, align=align,
                                                      capacity=cap)
        assert tot == e_tot
        assert np.array_equal(st, e_st)
        for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask",
                  "header_size"):
            assert np.array_equal(desc[f], e_d[f]), f
        assert np.array_equal(out[:tot], e_out[:tot])
    pl.close()


def test_pipeline_config2_reduced_digest():
    """1,024 x 64 KiB through host memory: the wire equals the reference's."""
    import hashlib
    g = golden("batch_digests.json")[0]
    n, fs = g["n_frames"], g["frame_size"]
    desc = W.uniform_batch(n, fs, g["key_seed"])
    payload_t, payload = pinned(n * fs)
    payload[:] = O.splitmix_words(g["payload_seed"], 0, n * fs // 8).view(np.uint8)
    wire_t, wire = pinned(g["wire_len"])
    pl = make_pipeline(chunk_bytes=8 << 20, max_frames=4096, depth=3)
    tot = pl.serialize(payload_t.data_ptr(), desc, wire_t.data_ptr(), wire.size)
    assert tot == g["wire_len"]
    if hashlib.sha256(wire[:tot].tobytes()).hexdigest() != g["wire_sha256"]:
        # say where: the keys drawn, then the bytes against the oracle's wire
        exp, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
        keys_ok = hashlib.sha256(exp.tobytes()).hexdigest() == g["wire_sha256"]
        bad = np.nonzero(wire[:tot] != exp)[0]
        frames = np.unique(np.searchsorted(desc["wire_off"], bad, side="right") - 1)
        pytest.fail(f"wire differs: keys as the reference's {keys_ok}, {bad.size} bytes, "
                    f"first at {bad[:4].tolist()}, frames {frames[:16].tolist()} "
                    f"({frames.size} in all)")
    back_t, back = pinned(n * fs)
    d2, st, ptot = pl.deserialize(wire_t.data_ptr(), tot, desc["wire_off"], back_t.data_ptr(),
                                  back.size)
    pl.close()
    assert ptot == n * fs and (st == 0).all()
    assert np.array_equal(back, payload)


@pytest.mark.parametrize("cut", [None, -1, -70000])
def test_pipeline_receive_indexes_then_deserializes(cut):
    """cfws_pipeline_receive: the host receive-loop walk, then the chunked
    device deserialize -- equal to the oracle's walk + batch deserialize,
    with a trailing partial frame (MORE_DATA) and an invalid frame (-7001)."""
    rng = random.Random(99)
    frames = [O.serialize_keyed(rng.random() < .7, rng.choice([0, 1, 2, 9]), rng.random() < .6,
                                rng.getrandbits(32),
                                rng.randbytes(rng.choice([0, 3, 125, 126, 5000, 70000])))
              for _ in range(600)]
    raw = b"".join(frames)
    if cut is not None:
        raw = raw[:cut]
    if cut == -70000:
        raw = raw[:len(raw) // 2] + b"\xf0\x00" + raw[len(raw) // 2:]
    wire_t, wire = pinned(len(raw))
    wire[:len(raw)] = np.frombuffer(raw, np.uint8)
    e_st, e_con, e_stop = O.index_stream(wire[:len(raw)], 0, len(raw))
    e_out, e_d, e_status, e_tot = O.deserialize_batch(wire[:len(raw)], e_st, align=16)
    out_t, out = pinned(e_tot + 64)
    pl = make_pipeline(chunk_bytes=1 << 20, max_frames=256, depth=3)
    desc, st, consumed, stop, tot = pl.receive(wire_t.data_ptr(), 0, len(raw), out_t.data_ptr(),
                                               out.size, max_frames=1000)
    pl.close()
    assert (consumed, stop) == (e_con, e_stop)
    assert len(desc) == len(e_st) and np.array_equal(desc["wire_off"], e_st)
    assert tot == e_tot and (st == 0).all()
    assert np.array_equal(desc["payload_off"], e_d["payload_off"])
    assert np.array_equal(out[:tot], e_out[:tot])


@pytest.mark.parametrize("max_frames,cut", [(4100, 0), (5000, 0), (2048, 0), (4999, 3), (0, 0)])
def test_pipeline_receive_walk_in_steps(max_frames, cut):
    """cfws_pipeline_receive walks the buffer a step (2,048 frames) ahead of
    the chunks; the walk's end equals one cfws_index_frames call over the whole
    buffer: the frame limit (CFWS_INDEX_FULL only when a COMPLETE frame
    follows), a cut last frame (MORE_DATA), consumed bytes, and the payloads."""
    rng = random.Random(max_frames + cut)
    frames = [O.serialize_keyed(True, 2, rng.random() < .6, rng.getrandbits(32),
                                rng.randbytes(rng.choice([0, 1, 9, 125, 126, 700])))
              for _ in range(5000)]
    raw = b"".join(frames)
    raw = raw[:len(raw) - cut]
    wire_t, wire = pinned(len(raw))
    wire[:len(raw)] = np.frombuffer(raw, np.uint8)
    e_st, e_con, e_stop = cfws.index_frames(wire[:len(raw)], 0, len(raw), max_starts=max_frames)
    e_out, e_d, e_status, e_tot = O.deserialize_batch(wire[:e_con], e_st, align=16)
    out_t, out = pinned(len(raw) + 16 * 5000 + 64)
    pl = make_pipeline(chunk_bytes=1 << 20, max_frames=700, depth=3)
    desc, st, consumed, stop, tot = pl.receive(wire_t.data_ptr(), 0, len(raw), out_t.data_ptr(),
                                               out.size, max_frames=max_frames)
    pl.close()
    assert (consumed, stop) == (e_con, e_stop)
    assert len(desc) == len(e_st) and np.array_equal(desc["wire_off"], e_st)
    assert tot == e_tot and np.array_equal(st, e_status)
    assert np.array_equal(out[:tot], e_out[:tot])


def _h2_batch(rng, n, sizes, payload_len):
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice(sizes)
        d[i] = (rng.randrange(0, payload_len - sz), 0, sz, rng.getrandbits(32), 1,
                rng.choice([1, 2, 9]), rng.random() < .7, 0)
    return d


@pytest.mark.parametrize("chunk,depth,S", [(1 << 17, 1, 16384), (1 << 17, 3, 100), (1 << 20, 2, 16),
                                           (1 << 20, 3, 16384)])
def test_pipeline_h2_serialize_matches_oracle(chunk, depth, S):
    """WS frames -> HTTP/2 DATA frames through host memory: the stream equals
    the oracle's co_http2_stream_send_ws_frame restatement byte for byte."""
    rng = random.Random(chunk + depth + S)
    payload_t, payload = pinned(1 << 20)
    payload[:] = O.fill_splitmix(1 << 20, S, 0)
    d = _h2_batch(rng, 1500, [0, 1, 125, 126, 999, 16376, 16384, 40000, 70000], 1 << 20)
    exp, exp_d = O.h2_serialize_batch(payload, d.copy(), 5, S)
    out_t, out = pinned(len(exp) + 64)
    pl = make_pipeline(chunk_bytes=chunk, max_frames=400, depth=depth)
    tot = pl.h2_serialize(payload_t.data_ptr(), d, out_t.data_ptr(), out.size, 5, S)
    pl.close()
    assert tot == len(exp)
    assert np.array_equal(d["header_size"], exp_d["header_size"])
    assert np.array_equal(out[:tot], exp)


@pytest.mark.parametrize("chunk,depth,S,align", [(1 << 18, 1, 16384, 16), (1 << 18, 3, 100, 1),
                                                 (1 << 20, 2, 13, 16), (1 << 20, 3, 16384, 64)])
def test_pipeline_h2_deserialize_matches_oracle(chunk, depth, S, align):
    """DATA frames -> pooled messages -> payloads through host memory, cut
    into chunks only where no message is open: HTTP/2 statuses, message
    descriptors and statuses, payloads and the total equal the oracle's, with
    corrupt headers, a non-DATA frame, an unterminated tail and a payload
    capacity cut. (A corrupt END_STREAM frame merges two messages: the
    chunks hold two of the largest.)"""
    rng = random.Random(chunk + depth + S + align)
    payload = O.fill_splitmix(1 << 20, 3, 0)
    d = _h2_batch(rng, 1200, [0, 5, 126, 999, 16376, 20000, 70000], 1 << 20)
    h2, _ = O.h2_serialize_batch(payload, d, 1, S)
    index = O.h2_index(h2)
    # a SETTINGS-like non-DATA frame between two DATA frames, an
    # unterminated message at the end (its last DATA frame's END_STREAM
    # cleared), and a few corrupt lengths
    k = int(index[len(index) // 3])
    h2 = np.concatenate([h2[:k], np.array([0, 0, 0, 4, 0, 0, 0, 0, 0], np.uint8), h2[k:]])
    index = O.h2_index(h2)
    h2[int(index[-1]) + 4] &= 0xFE
    for q in range(7, len(index) - 1, 211):
        h2[int(index[q])] = 0xFF                 # length > max_frame_size: PARSE_ERROR
    h2_t, h2_np = pinned(len(h2))
    h2_np[:len(h2)] = h2
    full = len(h2) + align * len(index) + 64
    pl = make_pipeline(chunk_bytes=chunk, max_frames=12000, depth=depth)
    for cap in (full, full // 3):
        out_t, out = pinned(cap)
        st, md, ms, tot = pl.h2_deserialize(h2_t.data_ptr(), len(h2), index, out_t.data_ptr(), cap,
                                            S=S, align=align)
        e = O.h2_deserialize_batch(h2, index, S, O.DEFAULT_MAX_PAYLOAD, align, None, cap)
        assert np.array_equal(st, e["h2_status"])
        assert len(md) == e["n_msg"] and tot == e["total"]
        assert np.array_equal(ms, e["msg_status"])
        for f in ("payload_off", "wire_off", "payload_size", "mask_key", "fin", "opcode", "mask",
                  "header_size"):
            assert np.array_equal(md[f], e["msg_desc"][f]), (cap, f)
        assert np.array_equal(out[:tot], e["payload"][:tot]), cap
    pl.close()
