#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REFERENCE codec itself.

Runs coldforce's own co_ws_frame_serialize / co_ws_frame_deserialize,
compiled in place from /root/reference by oracle/Makefile (`make -C oracle
ref` -> oracle/_ref/libcfws_ref.so). Only this container has the reference;
the committed JSON files are the data the GPU box checks against.

Fixtures (inputs + expected outputs):
  rfc6455_kat.json      RFC 6455 section 5.7 examples, decoded by the reference
  serialize_cases.json  boundary payload sizes x mask x fin/opcode x seed:
                        wire bytes (hex when small, SHA-256 always)
  deserialize_cases.json  decode results incl. truncations, invalid opcodes,
                        size limits, concatenated frames, non-minimal lengths
  keys.json             mask-key stream after srandom(seed)
  batch_digests.json    SHA-256 of whole serialized batches (config 2 full size)
  small_batch_digests.json  SHA-256 of the wire and of the reference's own
                        deserialize output for the small-frame batches the
                        bench quotes (4 M x 1 KiB TEXT, 16 M x 256 B BINARY)
  handshake_cases.json  Sec-WebSocket-Accept keys (co_sha1.c + co_base64.c)
  h2_echo_digests.json  DATA frames the stock HTTP/2 echo pair (the reference's
                        co_http2_stream.c send split and pooling) put on the wire
                        for WS frames of 16,376-65,536 B (--only h2echo)
  index_cases.json      receive-loop frame indexing (co_ws_server.c:107-169 around
                        the reference's co_ws_frame_deserialize): frame starts,
                        consumed index, stop code per connection stream

Payload bytes are synthetic: splitmix64 stream (oracle.fill_splitmix).
Usage: python tests/golden/make_golden.py [--skip-full]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SIZES = [0, 1, 3, 4, 5, 124, 125, 126, 127, 128, 65535, 65536, 65537, 1 << 20]
HEX_LIMIT = 300


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def dump(name: str, obj) -> None:
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1)
        f.write("\n")
    print("wrote", name)


def rfc6455(R):
    cases = [
        ("single-frame unmasked text", "810548656c6c6f"),
        ("single-frame masked text", "818537fa213d7f9f4d5158"),
        ("fragment 1 of unmasked text", "010348656c"),
        ("fragment 2 of unmasked text", "80026c6f"),
        ("unmasked ping", "890548656c6c6f"),
        ("masked pong", "8a8537fa213d7f9f4d5158"),
        ("256-byte unmasked binary", "827e0100" + "ab" * 256),
        ("65536-byte unmasked binary", "827f0000000000010000" + "cd" * 65536),
    ]
    out = []
    for name, hx in cases:
        raw = bytes.fromhex(hx)
        r = O.ref_deserialize(R, raw)
        out.append(dict(name=name, wire=hx if len(raw) <= HEX_LIMIT else None,
                        wire_sha256=sha(raw), wire_len=len(raw),
                        wire_spec=None if len(raw) <= HEX_LIMIT else hx[:20] + "+repeat",
                        rc=r["rc"], index=r["index"], fin=r["fin"], opcode=r["opcode"],
                        payload_size=r["payload_size"],
                        payload_hex=None if r["payload"] is None or len(r["payload"]) > HEX_LIMIT
                        else r["payload"].hex(),
                        payload_sha256=None if r["payload"] is None else sha(r["payload"])))
    return out


def serialize_cases(R):
    out = []
    variants = [(True, 0x2), (False, 0x0), (True, 0x1), (True, 0x9), (True, 0x7f), (False, 0xff)]
    for seed in (1, 1234):
        for n in SIZES:
            for mask in (False, True):
                for fin, op in variants:
                    if n >= 65536 and (fin, op) not in [(True, 0x2), (False, 0x0)]:
                        continue
                    base = n * 8
                    data = O.fill_splitmix(n, 0x5EEDF00D, base).tobytes()
                    O.srandom(R, seed)
                    w = O.ref_serialize(R, fin, op, mask, data)
                    out.append(dict(seed=seed, n=n, mask=mask, fin=fin, opcode=op,
                                    payload_seed=0x5EEDF00D, payload_byte_base=base,
                                    header_hex=w[:O.header_size(n, mask)].hex(),
                                    wire_hex=w.hex() if len(w) <= HEX_LIMIT else None,
                                    wire_len=len(w), wire_sha256=sha(w)))
    return out


def deserialize_cases(R):
    M = O.DEFAULT_MAX_PAYLOAD
    cases = []

    def add(name, wire: bytes, index=0, max_payload=M):
        r = O.ref_deserialize(R, wire, index, max_payload)
        p = r["payload"]
        cases.append(dict(name=name, wire_hex=wire.hex() if len(wire) <= 4096 else None,
                          wire_len=len(wire), wire_sha256=sha(wire),
                          wire_spec=None, index=index, max_payload=max_payload,
                          rc=r["rc"], index_out=r["index"], fin=r["fin"], opcode=r["opcode"],
                          payload_size=r["payload_size"], payload_is_null=p is None,
                          payload_hex=None if p is None or len(p) > 4096 else p.hex(),
                          payload_sha256=None if p is None else sha(p)))

    O.srandom(R, 77)
    masked300 = O.ref_serialize(R, True, 2, True, bytes(range(256)) + bytes(44))
    plain70k = O.ref_serialize(R, True, 2, False, b"\x5a" * 70000)
    add("masked 300 B", masked300)
    for cut in (2, 3, 4, 5, 7, 8, 100, len(masked300) - 1):
        add(f"masked 300 B truncated to {cut}", masked300[:cut])
    add("126-length header only", bytes([0x82, 0x7E]))
    add("127-length header, 7 of 8 length bytes", bytes([0x82, 0x7F]) + bytes(7))
    add("127-length header complete, no payload", bytes([0x82, 0x7F, 0, 0, 0, 0, 0, 1, 0, 0]))
    add("masked, key truncated", bytes([0x81, 0x85, 0x37, 0xFA, 0x21]))
    for b0 in (0xF2, 0xC1, 0xA1, 0x91, 0x47, 0x48, 0x10):
        add(f"b0=0x{b0:02x} (RSV bits / HTTP text)", bytes([b0, 0x05]) + b"Hello")
    for op in (3, 7, 0xB, 0xF):
        add(f"reserved opcode {op}", bytes([0x80 | op, 0x03]) + b"abc")
    add("zero-length masked", bytes([0x89, 0x80, 1, 2, 3, 4]))
    add("zero-length unmasked", bytes([0x8A, 0x00]))
    add("non-minimal 126 length of 5", bytes([0x81, 0x7E, 0x00, 0x05]) + b"Hello")
    add("non-minimal 127 length of 5", bytes([0x81, 0x7F]) + (5).to_bytes(8, "big") + b"Hello")
    add("64-bit length MSB set", bytes([0x82, 0x7F, 0x80, 0, 0, 0, 0, 0, 0, 1]) + b"xyz")
    add("length 33554433 header only (MORE_DATA before TOO_BIG)",
        bytes([0x82, 0x7F]) + (M + 1).to_bytes(8, "big"))
    two = bytes([0x81, 0x01, 0x41]) + bytes([0x82, 0x85, 1, 2, 3, 4]) + bytes(5)
    add("two frames, first", two, 0)
    add("two frames, second", two, 3)
    add("limit 300, payload 300", masked300, 0, 300)
    add("limit 299, payload 300 (TOO_BIG)", masked300, 0, 299)
    add("plain 70000 B", plain70k)
    add("plain 70000 B, limit 69999", plain70k, 0, 69999)
    # Full 33,554,433-byte payload -> DATA_TOO_BIG (described, not stored).
    big = bytes([0x82, 0x7F]) + (M + 1).to_bytes(8, "big") + bytes(M + 1)
    r = O.ref_deserialize(R, big)
    cases.append(dict(name="zero payload of 33554433 B (TOO_BIG)", wire_hex=None,
                      wire_spec="827f" + (M + 1).to_bytes(8, "big").hex() + "+zeros",
                      wire_len=len(big), wire_sha256=sha(big), index=0, max_payload=M,
                      rc=r["rc"], index_out=r["index"], fin=r["fin"], opcode=r["opcode"],
                      payload_size=r["payload_size"], payload_is_null=r["payload"] is None,
                      payload_hex=None, payload_sha256=None))
    return cases


def keys(R):
    out = {}
    for seed in (1, 2, 1234, 0x5EED):
        O.srandom(R, seed)
        ks = []
        for _ in range(16):
            w = O.ref_serialize(R, True, 2, True, b"")
            ks.append(w[2:6].hex())
        out[str(seed)] = ks
    return out


def batch_digest(R, n_frames, frame_size, payload_seed, key_seed, chunk=1024):
    """Serialize n_frames frames through the reference, sequentially, one
    co_byte_array per frame (co_ws_send), hashing the concatenated wire."""
    h = hashlib.sha256()
    hp = hashlib.sha256()
    total = 0
    O.srandom(R, key_seed)
    for c0 in range(0, n_frames, chunk):
        c1 = min(n_frames, c0 + chunk)
        words = O.splitmix_words(payload_seed, c0 * frame_size // 8, (c1 - c0) * frame_size // 8)
        arena = words.view(np.uint8)
        hp.update(arena.tobytes())
        for f in range(c1 - c0):
            w = O.ref_serialize(R, True, 2, True, arena[f * frame_size:(f + 1) * frame_size].tobytes())
            h.update(w)
            total += len(w)
    return dict(n_frames=n_frames, frame_size=frame_size, payload_seed=payload_seed,
                key_seed=key_seed, fin=True, opcode=2, mask=True, wire_len=total,
                wire_sha256=h.hexdigest(), payload_sha256=hp.hexdigest())


def small_batch_digest(R, n_frames, frame_size, payload_seed, key_seed, opcode, chunk=1 << 16):
    """n_frames x frame_size frames through the reference, in C
    (ref_serialize_run: co_ws_frame_serialize per frame, one byte array per
    frame as co_ws_send does), then the concatenated wire walked back
    through co_ws_frame_deserialize (ref_deserialize_run: the receive loop);
    SHA-256 of the wire and of the reference's unmasked payloads."""
    import ctypes as C
    ser, de = R.ref_serialize_run, R.ref_deserialize_run
    ser.argtypes = [C.c_void_p, C.c_ulonglong, C.c_ulonglong, C.c_int, C.c_ubyte, C.c_int,
                    C.c_void_p, C.c_ulonglong]
    ser.restype = C.c_longlong
    de.argtypes = [C.c_void_p, C.c_ulonglong, C.c_void_p, C.c_ulonglong,
                   C.POINTER(C.c_ulonglong)]
    de.restype = C.c_longlong
    hw, hp, ha = hashlib.sha256(), hashlib.sha256(), hashlib.sha256()
    total = 0
    O.srandom(R, key_seed)
    wire = np.empty(chunk * (frame_size + 14), np.uint8)
    back = np.empty(chunk * frame_size, np.uint8)
    for c0 in range(0, n_frames, chunk):
        c = min(n_frames, c0 + chunk) - c0
        arena = O.splitmix_words(payload_seed, c0 * frame_size // 8, c * frame_size // 8).view(np.uint8)
        ha.update(arena.tobytes())
        w = ser(arena.ctypes.data, c, frame_size, 1, opcode, 1, wire.ctypes.data, wire.size)
        assert w > 0, w
        hw.update(wire[:w].tobytes())
        total += w
        used = C.c_ulonglong(0)
        k = de(wire.ctypes.data, w, back.ctypes.data, back.size, C.byref(used))
        assert k == c and used.value == c * frame_size, (k, used.value)
        hp.update(back[:used.value].tobytes())
    assert ha.hexdigest() == hp.hexdigest()
    return dict(n_frames=n_frames, frame_size=frame_size, payload_seed=payload_seed,
                key_seed=key_seed, fin=True, opcode=opcode, mask=True, wire_len=total,
                wire_sha256=hw.hexdigest(), payload_sha256=hp.hexdigest())


def zipf_digest(R, target, seed, key_seed, ping_every=0):
    """Config 3: the Zipf message/fragment schedule (coldforce_amd.workloads,
    schedule only -- the keys come from the reference's own random() calls),
    serialized frame by frame through the reference."""
    from coldforce_amd import workloads as W
    desc, msgs = W.zipf_batch(target, seed, key_seed, ping_every=ping_every)
    arena_n = int(msgs["arena_bytes"])
    arena = O.splitmix_words(seed, 0, (arena_n + 7) // 8).view(np.uint8)[:arena_n]
    h = hashlib.sha256()
    total = 0
    O.srandom(R, key_seed)
    for d in desc:
        o, n = int(d["payload_off"]), int(d["payload_size"])
        w = O.ref_serialize(R, bool(d["fin"]), int(d["opcode"]), True, arena[o:o + n].tobytes())
        h.update(w)
        total += len(w)
    return dict(kind="zipf", target_bytes=target, seed=seed, key_seed=key_seed,
                ping_every=ping_every, n_frames=len(desc), n_messages=len(msgs["len"]),
                first_message_sizes=[int(x) for x in msgs["len"][:16]],
                arena_bytes=arena_n, arena_sha256=hashlib.sha256(arena.tobytes()).hexdigest(),
                wire_len=total, wire_sha256=h.hexdigest())


def h2_cases(R):
    """WebSocket over HTTP/2 through the reference: co_ws_frame_serialize +
    co_http2_frame.c DATA frames (split as co_http2_stream_send_data does),
    DATA decode cases through co_http2_frame_deserialize, and message-level
    results composed from the reference's DATA decode, the pooling rule of
    co_http2_stream.c:550-608 and co_ws_frame_deserialize."""
    out = {"wrap": [], "recv": [], "messages": []}
    for S, sid in ((16384, 1), (100, 3)):
        O.srandom(R, 5)
        h2 = b""
        frames = []
        for n, fin, op in ((0, 1, 9), (5, 1, 1), (125, 0, 1), (126, 0, 0), (16376, 1, 0),
                           (16377, 1, 2), (65536, 1, 2), (100000, 1, 2)):
            data = O.fill_splitmix(n, 0x5EED0005, 8 * n).tobytes()
            ws = O.ref_serialize(R, bool(fin), op, True, data)
            h2 += O.ref_h2_send(R, ws, S, sid)
            frames.append(dict(n=n, fin=fin, opcode=op, payload_seed=0x5EED0005, payload_byte_base=8 * n))
        out["wrap"].append(dict(max_frame=S, sid=sid, key_seed=5, frames=frames, h2_len=len(h2),
                                h2_sha256=sha(h2)))

    def hdr(length, typ, flags, sid):
        return bytes([length >> 16 & 255, length >> 8 & 255, length & 255, typ, flags]) + \
            (sid & 0x7fffffff).to_bytes(4, "big")
    data = bytes(range(40))
    cases = [
        ("DATA", hdr(40, 0, 0, 1) + data),
        ("DATA END_STREAM", hdr(40, 0, 1, 1) + data),
        ("DATA padded 7", hdr(48, 0, 8 | 1, 1) + bytes([7]) + data + bytes(7)),
        ("DATA padded 0", hdr(41, 0, 8, 1) + bytes([0]) + data),
        ("DATA empty END_STREAM", hdr(0, 0, 1, 1)),
        ("8-byte header", hdr(40, 0, 0, 1)[:8]),
        ("payload truncated", hdr(40, 0, 0, 1) + data[:39]),
        ("length over max_frame_size", hdr(16385, 0, 0, 1) + bytes(16385)),
        ("PING", hdr(8, 6, 0, 0) + bytes(8)),
    ]
    for name, raw in cases:
        r = O.ref_h2_recv(R, raw, 0, 16384)
        out["recv"].append(dict(name=name, raw_hex=raw.hex(), rc=r["rc"], index=r["index"],
                                length=r["length"], type=r["type"], flags=r["flags"],
                                payload_hex=r["payload"].hex()))
    # messages: DATA frames -> pool until END_STREAM -> co_ws_frame_deserialize
    O.srandom(R, 6)
    stream = b""
    ws_msgs = [O.ref_serialize(R, True, 1, True, b"hello"),
               O.ref_serialize(R, True, 2, True, bytes(range(256)) * 150),
               O.ref_serialize(R, False, 2, True, bytes(300)),
               bytes([0x82, 0x85, 1, 2, 3, 4]) + b"ab",                # WS frame longer than its message
               O.ref_serialize(R, True, 9, False, b"")]
    for k, ws in enumerate(ws_msgs):
        if k == 2:   # one message split with padded DATA frames
            stream += hdr(100 + 1 + 3, 0, 8, 1) + bytes([3]) + ws[:100] + bytes(3)
            stream += hdr(len(ws) - 100, 0, 1, 1) + ws[100:]
        else:
            stream += O.ref_h2_send(R, ws, 16384 if k != 1 else 1000, 1)
    idx, pool, msgs = 0, b"", []
    while idx < len(stream):
        r = O.ref_h2_recv(R, stream, idx, 16384)
        assert r["rc"] == 0
        idx = r["index"]
        pool += r["payload"]
        if r["flags"] & 1:
            msgs.append(pool)
            pool = b""
    res = []
    for m in msgs:
        d = O.ref_deserialize(R, m, 0)
        res.append(dict(rc=d["rc"], fin=d["fin"], opcode=d["opcode"], payload_size=d["payload_size"],
                        payload_sha256=None if d["payload"] is None else sha(d["payload"][:-1]),
                        message_len=len(m)))
    out["messages"].append(dict(stream_hex=stream.hex(), max_frame=16384, results=res))
    return out


def h2_digest(R, n_frames, frame_size, payload_seed, key_seed, S=16384, sid=1):
    """Config 5: n_frames binary frames, client-masked, each carried in
    HTTP/2 DATA frames of at most S bytes, through the reference."""
    h = hashlib.sha256()
    total = 0
    O.srandom(R, key_seed)
    chunk = 1024
    for c0 in range(0, n_frames, chunk):
        c1 = min(n_frames, c0 + chunk)
        arena = O.splitmix_words(payload_seed, c0 * frame_size // 8,
                                 (c1 - c0) * frame_size // 8 + 1).view(np.uint8)
        for f in range(c1 - c0):
            ws = O.ref_serialize(R, True, 2, True, arena[f * frame_size:(f + 1) * frame_size].tobytes())
            h2 = O.ref_h2_send(R, ws, S, sid)
            h.update(h2)
            total += len(h2)
    return dict(n_frames=n_frames, frame_size=frame_size, payload_seed=payload_seed,
                key_seed=key_seed, max_frame=S, sid=sid, h2_len=total, h2_sha256=h.hexdigest())


H2_ECHO_SIZES = (16376, 16377, 40000, 65536)


def h2_echo_cases():
    """The reference's own HTTP/2 stream code on WS frames that span several
    DATA frames: the stock echo pair (oracle/_ref/ws_echo_stock, h2 mode:
    co_http2_stream_send_ws_frame -> co_http2_stream_send_data's split,
    co_http2_stream.c:933-1013, and the receiver's pooling, :550-608) sends
    `frames` TEXT frames of each size, client-masked with the srandom(seed)
    stream, and echoes them unmasked. The capture of each side gives the
    DATA frames (9-byte header + payload) that carried the WS frames: their
    count, the DATA payload sizes of one WS frame, and the SHA-256 of all of
    them back to back."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from echo_util import available, h2_data_frames, run_echo
    assert available("stock"), "oracle/_ref/ws_echo_stock not built"
    out = []
    for i, payload in enumerate(H2_ECHO_SIZES):
        frames, window, seed = 64, 8, 21 + i
        with tempfile.TemporaryDirectory() as tmp:
            r = run_echo("stock", "h2", frames, payload, window=window, seed=seed, capture_dir=tmp)
            assert r["client_rc"] == 0 and r["client"]["received"] == frames and r["client"]["bad_echo"] == 0
            case = dict(payload=payload, frames=frames, window=window, seed=seed, opcode=1, sid=1,
                        max_frame=16384)
            for side in ("client", "server"):
                with open(r["capture"][side], "rb") as f:
                    data = h2_data_frames(f.read(), preface=side == "client")
                raw = b"".join(d for _, d in data)
                per = len(data) // frames
                case[side] = dict(mask=side == "client", data_frames=len(data),
                                  end_stream=sum(1 for fl, _ in data if fl & 1),
                                  split=[len(d) - 9 for _, d in data[:per]], data_len=len(raw),
                                  data_sha256=sha(raw))
        out.append(case)
    return out


def index_cases(R):
    """Streams of reference-serialized frames, cut and corrupted the ways a
    receive buffer can be; the reference's loop gives starts/consumed/stop.
    Each distinct byte string is stored once (`blobs`); a case is a prefix of
    a blob, a receive index and a payload limit."""
    import random
    rng = random.Random(0x1D3)
    O.srandom(R, 4242)
    M = O.DEFAULT_MAX_PAYLOAD

    def frames(spec):
        return [O.ref_serialize(R, fin, op, mask, O.fill_splitmix(n, 0x1D3 + n).tobytes())
                for (fin, op, mask, n) in spec]

    base = frames([(1, 1, 1, 0), (1, 2, 1, 1), (0, 1, 0, 125), (1, 0, 1, 126), (1, 9, 0, 5),
                   (1, 2, 1, 65535), (1, 2, 0, 65536), (1, 8, 1, 2), (1, 2, 1, 70000),
                   (1, 10, 0, 0), (1, 2, 1, 300)])
    whole = b"".join(base)
    ends = [int(x) for x in np.cumsum([len(f) for f in base])]
    blobs = {"whole": whole,
             "whole+1": whole + b"\x82",
             "http": b"GET / HTTP/1.1\r\nHost: x\r\n\r\n",
             "rsv": whole[:ends[2]] + b"\xc2\x00" + whole[ends[2]:ends[4]],
             "msb64": whole[:ends[0]] + bytes([0x82, 0x7f, 0x80]) + bytes(7),
             "tiny": b"\x82\x00" * 300 + b"\x81\x01a" * 200}
    cases = [("empty", "whole", 0, 0, M), ("one byte", "whole", 1, 0, M),
             ("whole", "whole", len(whole), 0, M), ("trailing byte", "whole+1", len(whole) + 1, 0, M),
             ("receive index mid-buffer", "whole", len(whole), ends[2], M),
             ("receive index at end", "whole", len(whole), len(whole), M),
             ("http request", "http", None, 0, M), ("rsv bit after 3 frames", "rsv", None, 0, M),
             ("too big complete", "whole", len(whole), 0, 1000),
             ("too big incomplete (MORE_DATA first)", "whole", ends[4] + 5000, 0, 1000),
             ("64-bit length msb", "msb64", None, 0, M), ("tiny frames", "tiny", None, 0, M)]
    for k in (1, 3, 5, 8):
        for cut in (1, 2, 3, 4, 5, 9, 13, 14, 100):
            cases.append((f"cut {cut} B into frame {k}", "whole", ends[k - 1] + cut, 0, M))
    for t in range(24):
        spec = [(rng.random() < .7, rng.choice([0, 1, 2, 8, 9, 10, 3]), rng.random() < .5,
                 rng.choice([0, 1, 2, 7, 125, 126, 127, 1000, 4096] + ([65536] if t % 6 == 0 else [])))
                for _ in range(rng.randrange(1, 40))]
        w = b"".join(frames(spec))
        blobs[f"random {t}"] = w
        cut = len(w) if t % 3 == 0 else rng.randrange(0, len(w) + 1)
        cases.append((f"random {t}", f"random {t}", cut, 0, M))
    out = []
    for name, blob, cut, begin, mp in cases:
        data = blobs[blob][:cut] if cut is not None else blobs[blob]
        st, consumed, stop = O.ref_index_stream(R, data, begin, mp)
        out.append(dict(name=name, blob=blob, size=len(data), begin=begin, max_payload=mp,
                        starts=[int(x) for x in st], consumed=consumed, stop=stop))
    return dict(blobs={k: v.hex() for k, v in blobs.items()}, cases=out)


def handshake_cases(R):
    """Sec-WebSocket-Accept for keys of every shape through the reference's
    co_sha1.c + co_base64.c (lengths 0-300 cross SHA-1's one/two/three
    block padding boundaries: 55/56 and 119/120 bytes with the 36-byte GUID)."""
    import random
    rng = random.Random(0xACCE)
    keys = [b"dGhlIHNhbXBsZSBub25jZQ==", b""]                 # RFC 6455 1.3 example
    for n in [1, 2, 3, 16, 18, 19, 20, 24, 27, 28, 63, 64, 83, 84, 85, 100, 147, 148, 200, 300]:
        keys.append(bytes(rng.randrange(33, 127) for _ in range(n)))
    for _ in range(40):                                           # real-shaped nonces
        import base64
        keys.append(base64.b64encode(rng.randbytes(16)))
    return [dict(key_hex=k.hex(), accept=O.ref_ws_accept_key(R, k)) for k in keys]


SMALL_BATCHES = [(4 << 20, 1024, 1), (16 << 20, 256, 2), ((4 << 30) // 2048, 2048, 2),
                 ((4 << 30) // 3072, 3072, 2), ((4 << 30) // 3584, 3584, 1), (8 << 20, 512, 2)]


def small_batches(R, have=()):
    # the bench's payload / key seeds (bench.py PAYLOAD_SEED, KEY_SEED);
    # 1 KiB as TEXT (config 1's frames), 256 B and 512 B as BINARY; the
    # in-region send's range (payloads up to 3,584 B, round 4): 2 KiB and
    # 3 KiB batches of 4 GiB as the bench runs them (bench.py --frame-size:
    # 4 GiB // size frames), and payloads of exactly the bound. Entries
    # already in `have` (same frames, size, opcode) are kept, not recomputed.
    old = {(d["n_frames"], d["frame_size"], d["opcode"]): d for d in have}
    return [old.get((n, fs, op)) or small_batch_digest(R, n, fs, 0x5EED0002, 2, op)
            for n, fs, op in SMALL_BATCHES]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true", help="skip the 4 GiB config-2 digest")
    ap.add_argument("--only", help="regenerate one fixture family (e.g. index)")
    a = ap.parse_args()
    O.build(ref=True)
    R = O.ref_lib("O2")
    assert R is not None, "oracle/_ref not built (needs /root/reference)"
    if a.only == "index":
        dump("index_cases.json", index_cases(R))
        return
    if a.only == "small":
        path = os.path.join(OUT, "small_batch_digests.json")
        have = json.load(open(path)) if os.path.exists(path) else []
        dump("small_batch_digests.json", small_batches(R, have))
        return
    if a.only == "handshake":
        dump("handshake_cases.json", handshake_cases(R))
        return
    if a.only == "h2echo":
        dump("h2_echo_digests.json", h2_echo_cases())
        return
    dump("rfc6455_kat.json", rfc6455(R))
    dump("serialize_cases.json", serialize_cases(R))
    dump("deserialize_cases.json", deserialize_cases(R))
    dump("keys.json", keys(R))
    digests = [batch_digest(R, 1024, 65536, 0x5EED0002, 2),
               batch_digest(R, 4096, 1000, 0x5EED00AA, 9)]
    if not a.skip_full:
        digests.append(batch_digest(R, 65536, 65536, 0x5EED0002, 2))
    dump("batch_digests.json", digests)
    zipf = [zipf_digest(R, 64 << 20, 0x5EED0003, 3), zipf_digest(R, 8 << 20, 0x5EED0033, 33, ping_every=3)]
    if not a.skip_full:
        zipf.append(zipf_digest(R, 4 << 30, 0x5EED0003, 3))
    dump("zipf_digests.json", zipf)
    dump("h2_cases.json", h2_cases(R))
    h2d = [h2_digest(R, 1024, 16376, 0x5EED0005, 5), h2_digest(R, 1024, 65536, 0x5EED0005, 5)]
    if not a.skip_full:
        h2d += [h2_digest(R, 65536, 16376, 0x5EED0005, 5), h2_digest(R, 65536, 65536, 0x5EED0005, 5)]
    dump("h2_digests.json", h2d)
    dump("index_cases.json", index_cases(R))
    dump("handshake_cases.json", handshake_cases(R))
    dump("h2_echo_digests.json", h2_echo_cases())
    if not a.skip_full:
        dump("small_batch_digests.json", small_batches(R))


if __name__ == "__main__":
    main()
