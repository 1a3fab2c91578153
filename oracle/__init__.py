"""TEST INFRASTRUCTURE ONLY -- ctypes bindings for the parity checker.

``liboracle.so`` is the clean-room CPU restatement of coldforce's frame codec
(``oracle/cfws_oracle.c``); ``_ref/libcfws_ref*.so`` is the reference codec
itself, compiled in place from ``/root/reference`` by ``oracle/Makefile``
(absent on the GPU box unless built here first).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this package; ``coldforce_amd`` never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = {"O2": os.path.join(HERE, "_ref", "libcfws_ref.so"),
          "O0": os.path.join(HERE, "_ref", "libcfws_ref_O0.so")}

PARSE_COMPLETE = 0
PARSE_MORE_DATA = 1
ERROR_INVALID_FRAME = -7001
ERROR_DATA_TOO_BIG = -7005
ERROR_OUT_OF_MEMORY = -7006
DEFAULT_MAX_PAYLOAD = 32 * 1024 * 1024  # co_ws_config.h:15

# Same 32-byte layout as cfws_frame_desc_t (include/cfws.h) / orc_desc_t.
DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("wire_off", "<u8"),
                       ("payload_size", "<u8"), ("mask_key", "<u4"),
                       ("fin", "u1"), ("opcode", "u1"), ("mask", "u1"),
                       ("header_size", "u1")])
assert DESC_DTYPE.itemsize == 32

_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p
_u64 = C.c_uint64
_sz = C.c_size_t


def _ptr(a):
    return a.ctypes.data_as(_vp) if a is not None else None


def build(ref: bool = True) -> None:
    """Compile the restatement (and the reference when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build(ref=False)
        L = C.CDLL(ORACLE_SO)
        L.orc_serialize_keyed.argtypes = [C.c_bool, C.c_uint8, C.c_bool, C.c_uint32, _vp, _sz, _vp]
        L.orc_serialize_keyed.restype = _sz
        L.orc_header_size.argtypes = [_u64, C.c_bool]
        L.orc_header_size.restype = C.c_uint32
        L.orc_keys.argtypes = [C.c_uint32, _sz, _vp, _vp]
        L.orc_serialize_batch.argtypes = [_vp, _vp, _sz, _vp]
        L.orc_serialize_batch.restype = _u64
        L.orc_deserialize_batch.argtypes = [_vp, _u64, _vp, _sz, _u64, C.c_uint32, C.c_uint32,
                                            _vp, _vp, _vp, _u64]
        L.orc_deserialize_batch.restype = _u64
        L.orc_encode_headers.argtypes = [_vp, _sz, _vp, _u64]
        L.orc_parse_headers.argtypes = [_vp, _u64, _vp, _sz, _u64, _vp, _vp]
        L.orc_mask_batch.argtypes = [_vp, _vp, _sz, _vp, _u64]
        L.orc_unmask_batch.argtypes = [_vp, _vp, _vp, _sz, _vp, _u64]
        L.orc_index_frames.argtypes = [_vp, _u64, _u64, _vp, _sz, C.POINTER(_u64)]
        L.orc_index_frames.restype = _sz
        L.orc_fill_splitmix.argtypes = [_vp, _u64, _u64, _u64]
        L.orc_cpu_bench.argtypes = [_u64, _u64, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_cpu_bench.restype = C.c_int
        _bind_flat(L, "orc")
        _lib = L
    return _lib


def header_size(n: int, mask: bool) -> int:
    return lib().orc_header_size(n, mask)


def serialize_keyed(fin: bool, opcode: int, mask: bool, key: int, data: bytes) -> bytes:
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(len(data) + 16, dtype=np.uint8)
    n = lib().orc_serialize_keyed(fin, opcode, mask, key, _ptr(src), len(data), _ptr(out))
    return out[:n].tobytes()


def keys(seed: int, n: int, mask_flags=None) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint32)
    mf = None if mask_flags is None else np.ascontiguousarray(mask_flags, dtype=np.uint8)
    lib().orc_keys(seed, n, _ptr(mf), _ptr(out))
    return out


def serialize_batch(payload: np.ndarray, desc: np.ndarray):
    """Returns (wire bytes ndarray, desc with wire_off/header_size filled)."""
    desc = desc.copy()
    total = int(sum(int(d["payload_size"]) + header_size(int(d["payload_size"]), bool(d["mask"]))
                    for d in desc)) if len(desc) < 4096 else None
    if total is None:
        sizes = desc["payload_size"].astype(np.uint64)
        hs = 2 + np.where(sizes > 65535, 8, np.where(sizes > 125, 2, 0)) + 4 * (desc["mask"] != 0)
        total = int((sizes + hs.astype(np.uint64)).sum())
    wire = np.zeros(max(total, 1), dtype=np.uint8)
    pl = payload if payload.size else np.zeros(1, np.uint8)
    n = lib().orc_serialize_batch(_ptr(pl), _ptr(desc), len(desc), _ptr(wire))
    assert n == total
    return wire[:total], desc


DESERIALIZE_REASSEMBLE = 1


def deserialize_batch(wire: np.ndarray, starts: np.ndarray, align: int = 16,
                      max_payload: int = DEFAULT_MAX_PAYLOAD, capacity: int | None = None,
                      flags: int = 0):
    """Returns (payload arena, desc, status, total)."""
    starts = np.ascontiguousarray(starts, dtype=np.uint64)
    n = len(starts)
    if capacity is None:
        capacity = len(wire) + 16 * n + 16
    desc = np.zeros(n, dtype=DESC_DTYPE)
    status = np.zeros(n, dtype=np.int32)
    out = np.zeros(max(capacity, 1), dtype=np.uint8)
    w = wire if wire.size else np.zeros(1, np.uint8)
    total = lib().orc_deserialize_batch(_ptr(w), len(wire), _ptr(starts), n, max_payload,
                                        align, flags, _ptr(desc), _ptr(status), _ptr(out),
                                        capacity)
    return out, desc, status, int(total)


def encode_headers(desc: np.ndarray, wire: np.ndarray, capacity: int | None = None) -> np.ndarray:
    """Split op (include/cfws.h): headers at wire_off, in place in `wire`;
    returns desc with header_size set."""
    desc = desc.copy()
    cap = len(wire) if capacity is None else capacity
    lib().orc_encode_headers(_ptr(desc), len(desc), _ptr(wire), cap)
    return desc


def parse_headers(wire: np.ndarray, starts: np.ndarray, max_payload: int = DEFAULT_MAX_PAYLOAD,
                  wire_size: int | None = None):
    starts = np.ascontiguousarray(starts, dtype=np.uint64)
    desc = np.zeros(len(starts), dtype=DESC_DTYPE)
    status = np.zeros(len(starts), dtype=np.int32)
    size = len(wire) if wire_size is None else wire_size
    w = wire if wire.size else np.zeros(1, np.uint8)
    lib().orc_parse_headers(_ptr(w), size, _ptr(starts), len(starts), max_payload, _ptr(desc),
                            _ptr(status))
    return desc, status


def mask_batch(payload: np.ndarray, desc: np.ndarray, wire: np.ndarray,
               capacity: int | None = None) -> None:
    """Split op: masked payloads into `wire` in place (headers untouched)."""
    cap = len(wire) if capacity is None else capacity
    pl = payload if payload.size else np.zeros(1, np.uint8)
    lib().orc_mask_batch(_ptr(pl), _ptr(np.ascontiguousarray(desc)), len(desc), _ptr(wire), cap)


def unmask_batch(wire: np.ndarray, desc: np.ndarray, status, payload: np.ndarray,
                 capacity: int | None = None) -> None:
    """Split op: unmasked payloads into `payload` in place."""
    cap = len(payload) if capacity is None else capacity
    st = None if status is None else np.ascontiguousarray(status, dtype=np.int32)
    lib().orc_unmask_batch(_ptr(wire), _ptr(np.ascontiguousarray(desc)), _ptr(st), len(desc),
                           _ptr(payload), cap)


def index_frames(wire: np.ndarray, max_frames: int, max_payload: int = DEFAULT_MAX_PAYLOAD):
    starts = np.zeros(max(max_frames, 1), dtype=np.uint64)
    consumed = _u64(0)
    w = wire if wire.size else np.zeros(1, np.uint8)
    k = lib().orc_index_frames(_ptr(w), len(wire), max_payload, _ptr(starts), max_frames,
                               C.byref(consumed))
    return starts[:k], int(consumed.value)


def index_stream(buf: np.ndarray, begin: int = 0, end: int | None = None,
                 max_payload: int = DEFAULT_MAX_PAYLOAD):
    """One connection's receive loop over buf[begin, end) (orc_index_stream):
    (starts, consumed, stop)."""
    end = len(buf) if end is None else end
    f = lib().orc_index_stream
    f.argtypes = [_vp, _u64, _u64, _u64, _vp, _sz, C.POINTER(_u64), C.POINTER(C.c_int32)]
    f.restype = _sz
    b = buf if buf.size else np.zeros(1, np.uint8)
    cap = max((end - begin) // 2 + 1, 1)
    starts = np.zeros(cap, dtype=np.uint64)
    consumed, stop = _u64(0), C.c_int32(0)
    k = f(_ptr(b), begin, end, max_payload, _ptr(starts), cap, C.byref(consumed), C.byref(stop))
    return starts[:k], int(consumed.value), int(stop.value)


def ws_accept_key(key: bytes) -> str:
    """base64(SHA-1(key || GUID)) -- co_ws_create_base64_accept_key."""
    f = lib().orc_ws_accept_key
    f.argtypes = [C.c_char_p, _u64, C.c_char_p]
    f.restype = None
    out = C.create_string_buffer(29)
    f(key, len(key), out)
    return out.value.decode()


def fill_splitmix(n_bytes: int, seed: int, byte_base: int = 0) -> np.ndarray:
    out = np.zeros(max(n_bytes, 1), dtype=np.uint8)
    lib().orc_fill_splitmix(_ptr(out), n_bytes, seed, byte_base)
    return out[:n_bytes]


def splitmix_words(seed: int, first_word: int, n_words: int) -> np.ndarray:
    """Vectorised numpy splitmix64 (same function as orc_fill_splitmix)."""
    i = np.arange(first_word, first_word + n_words, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def cpu_bench(n_frames: int, frame_size: int, threads: int, iters: int, kind: str = "port"):
    """Time per-frame serialize(mask)+deserialize. Returns (mask_s, unmask_s)."""
    if kind == "port":
        L, fn = lib(), "orc_cpu_bench"
    else:
        L, fn = ref_lib(kind[len("reference"):].strip("_-") or "O2"), "ref_cpu_bench"
        if L is None:
            raise FileNotFoundError("oracle/_ref not built")
    f = getattr(L, fn)
    f.argtypes = [_u64, _u64, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    f.restype = C.c_int
    ms, us = C.c_double(0), C.c_double(0)
    rc = f(n_frames, frame_size, threads, iters, C.byref(ms), C.byref(us))
    if rc != 0:
        raise RuntimeError(f"cpu bench failed rc={rc}")
    return ms.value, us.value


def cpu_h2_bench(n_frames: int, frame_size: int, max_frame: int, threads: int, iters: int,
                 opt: str = "O2"):
    """Config 5 on the host through the reference compiled in place
    (oracle/_ref, ref_h2_cpu_bench): per WS frame co_ws_frame_serialize(mask)
    + the DATA split of co_http2_stream_send_data through co_http2_frame.c
    (send), then co_http2_frame_deserialize + the stream's pooling +
    co_ws_frame_deserialize (receive). Returns (send_s, recv_s)."""
    L = ref_lib(opt)
    if L is None:
        raise FileNotFoundError("oracle/_ref not built")
    f = L.ref_h2_cpu_bench
    f.argtypes = [_u64, _u64, C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_double),
                  C.POINTER(C.c_double)]
    f.restype = C.c_int
    ss, rs = C.c_double(0), C.c_double(0)
    rc = f(n_frames, frame_size, max_frame, threads, iters, C.byref(ss), C.byref(rs))
    if rc != 0:
        raise RuntimeError(f"h2 cpu bench failed rc={rc}")
    return ss.value, rs.value


# ---- the reference itself (oracle/_ref), when built -------------------------


class _Flat:
    """Uniform per-frame API over either library (prefix orc_ or ref_)."""

    def __init__(self, L, prefix):
        self.srandom = getattr(L, prefix + "_srandom")
        self.serialize = getattr(L, prefix + "_serialize" + ("_flat" if prefix == "orc" else ""))
        self.deserialize = getattr(L, prefix + "_deserialize" + ("_flat" if prefix == "orc" else ""))


def _bind_flat(L, prefix):
    f = _Flat(L, prefix)
    f.srandom.argtypes = [C.c_uint]
    f.srandom.restype = None
    f.serialize.argtypes = [C.c_int, C.c_ubyte, C.c_int, _vp, C.c_ulonglong, _vp, C.c_ulonglong]
    f.serialize.restype = C.c_longlong
    f.deserialize.argtypes = [_vp, C.c_ulonglong, C.POINTER(C.c_ulonglong), C.c_ulonglong,
                              C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_ulonglong),
                              C.POINTER(C.c_int), _vp, C.c_ulonglong]
    f.deserialize.restype = C.c_int
    L.flat = f

_ref = {}


def cpu_accept_bench(raw: np.ndarray, off: np.ndarray, threads: int, iters: int,
                     kind: str = "port") -> float:
    """Seconds for `iters` passes of co_ws_create_base64_accept_key over every
    key raw[off[i]:off[i+1]] on `threads` host threads (kind "reference":
    the reference's co_sha1.c + co_base64.c compiled in place)."""
    L, fn = (lib(), "orc_accept_bench") if kind == "port" else (ref_lib("O2"), "ref_accept_bench")
    if L is None:
        raise FileNotFoundError("oracle/_ref not built")
    f = getattr(L, fn)
    f.argtypes = [_vp, _vp, _u64, C.c_int, C.c_int, C.POINTER(C.c_double)]
    f.restype = C.c_int
    o = np.ascontiguousarray(off, dtype=np.uint64)
    sec = C.c_double(0)
    if f(_ptr(raw), _ptr(o), len(o) - 1, threads, iters, C.byref(sec)) != 0:
        raise RuntimeError("accept bench failed")
    return sec.value


def cpu_index_bench(buf: np.ndarray, begin: np.ndarray, end: np.ndarray, max_per_conn: int,
                    threads: int) -> tuple[float, int]:
    """The receive-loop walk (orc_index_stream) over every connection
    buf[begin[c], end[c]) on `threads` host threads: (seconds, frames)."""
    f = lib().orc_index_bench
    f.argtypes = [_vp, _vp, _vp, _u64, _u64, C.c_int, C.POINTER(C.c_double), C.POINTER(_u64)]
    f.restype = C.c_int
    b = np.ascontiguousarray(begin, dtype=np.uint64)
    e = np.ascontiguousarray(end, dtype=np.uint64)
    sec, frames = C.c_double(0), _u64(0)
    if f(_ptr(buf), _ptr(b), _ptr(e), len(b), max_per_conn, threads, C.byref(sec), C.byref(frames)) != 0:
        raise RuntimeError("index bench failed")
    return sec.value, frames.value


def ref_lib(opt: str = "O2"):
    if opt not in _ref:
        path = REF_SO[opt]
        if not os.path.exists(path):
            return None
        L = C.CDLL(path)
        _bind_flat(L, "ref")
        _ref[opt] = L
    return _ref[opt]


def srandom(L, seed: int) -> None:
    L.flat.srandom(seed)


def ref_serialize(L, fin: bool, opcode: int, mask: bool, data: bytes) -> bytes:
    """co_ws_frame_serialize through library L (oracle lib() or ref_lib())."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(len(data) + 16, dtype=np.uint8)
    n = L.flat.serialize(int(fin), opcode, int(mask), _ptr(src), len(data), _ptr(out), out.size)
    assert n >= 0, n
    return out[:n].tobytes()


def ref_deserialize(L, data: bytes, index: int = 0, max_payload: int = DEFAULT_MAX_PAYLOAD):
    """co_ws_frame_deserialize through library L. Returns dict(rc, index, fin, opcode, payload_size, payload|None)."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(len(data) + 2, dtype=np.uint8)
    idx = C.c_ulonglong(index)
    fin, op, isnull = C.c_int(), C.c_int(), C.c_int()
    psz = C.c_ulonglong()
    rc = L.flat.deserialize(_ptr(src), len(data), C.byref(idx), max_payload, C.byref(fin),
                           C.byref(op), C.byref(psz), C.byref(isnull), _ptr(out), out.size)
    payload = None
    if rc == 0 and not isnull.value:
        payload = out[:psz.value + 1].tobytes()  # includes the NUL terminator
    return dict(rc=rc, index=idx.value, fin=bool(fin.value), opcode=op.value,
                payload_size=psz.value, payload=payload)


# ---- WebSocket over HTTP/2 ----------------------------------------------------

def _bind_h2():
    L = lib()
    if not hasattr(L, "_h2_bound"):
        L.orc_h2_send.argtypes = [_vp, _u64, C.c_uint32, C.c_uint32, _vp]
        L.orc_h2_send.restype = _u64
        L.orc_h2_serialize_batch.argtypes = [_vp, _vp, _sz, C.c_uint32, C.c_uint32, _vp, _vp]
        L.orc_h2_serialize_batch.restype = _u64
        L.orc_h2_deserialize_batch.argtypes = [_vp, _u64, _vp, _sz, C.c_uint32, _vp, _vp, _u64,
                                               _u64, C.c_uint32, _vp, _vp, _vp, _u64,
                                               C.POINTER(_u64)]
        L.orc_h2_deserialize_batch.restype = _u64
        L._h2_bound = True
    return L


def h2_frames_bound(ws_len: int, S: int) -> int:
    return 9 * (ws_len // S + 2) + ws_len


def h2_serialize_batch(payload: np.ndarray, desc: np.ndarray, sid: int = 1, S: int = 16384):
    """Returns (h2 bytes, desc with header_size filled)."""
    L = _bind_h2()
    desc = desc.copy()
    sizes = desc["payload_size"].astype(np.uint64)
    w = sizes + 14
    bound = int((w + 9 * (w // S + 1)).sum()) + 64
    out = np.zeros(bound, dtype=np.uint8)
    tmp = np.zeros(int(w.max()) + 16 if len(w) else 16, dtype=np.uint8)
    pl = payload if payload.size else np.zeros(1, np.uint8)
    n = L.orc_h2_serialize_batch(_ptr(pl), _ptr(desc), len(desc), sid, S, _ptr(tmp), _ptr(out))
    return out[:n], desc


def h2_deserialize_batch(h2: np.ndarray, index: np.ndarray, S: int = 16384,
                         max_payload: int = DEFAULT_MAX_PAYLOAD, align: int = 16,
                         pool_capacity: int | None = None, payload_capacity: int | None = None):
    """Returns dict(h2_status, pool, msg_desc, msg_status, payload, total, n_msg)."""
    L = _bind_h2()
    index = np.ascontiguousarray(index, dtype=np.uint64)
    n = len(index)
    pool_capacity = len(h2) if pool_capacity is None else pool_capacity
    payload_capacity = len(h2) + 16 * n + 16 if payload_capacity is None else payload_capacity
    h2_status = np.zeros(n, dtype=np.int32)
    pool = np.zeros(max(pool_capacity, 1), dtype=np.uint8)
    msg_desc = np.zeros(max(n, 1), dtype=DESC_DTYPE)
    msg_status = np.zeros(max(n, 1), dtype=np.int32)
    payload = np.zeros(max(payload_capacity, 1), dtype=np.uint8)
    n_msg = _u64(0)
    h = h2 if h2.size else np.zeros(1, np.uint8)
    total = L.orc_h2_deserialize_batch(_ptr(h), len(h2), _ptr(index), n, S, _ptr(h2_status),
                                       _ptr(pool), pool_capacity, max_payload, align,
                                       _ptr(msg_desc), _ptr(msg_status), _ptr(payload),
                                       payload_capacity, C.byref(n_msg))
    m = n_msg.value
    return dict(h2_status=h2_status, pool=pool, msg_desc=msg_desc[:m], msg_status=msg_status[:m],
                payload=payload, total=int(total), n_msg=m)


def h2_index(h2: np.ndarray) -> np.ndarray:
    """Frame starts of a well-formed HTTP/2 frame stream (sequential walk)."""
    starts, p, n = [], 0, len(h2)
    while p + 9 <= n:
        starts.append(p)
        p += 9 + (int(h2[p]) << 16 | int(h2[p + 1]) << 8 | int(h2[p + 2]))
    return np.array(starts, dtype=np.uint64)


def ref_h2_send(R, ws: bytes, S: int = 16384, sid: int = 1) -> bytes:
    f = R.ref_h2_send
    f.argtypes = [_vp, C.c_ulonglong, C.c_uint, C.c_uint, _vp, C.c_ulonglong]
    f.restype = C.c_longlong
    src = np.frombuffer(ws, dtype=np.uint8) if ws else np.zeros(1, np.uint8)
    out = np.zeros(len(ws) + 9 * (len(ws) // S + 2), dtype=np.uint8)
    k = f(_ptr(src), len(ws), S, sid, _ptr(out), out.size)
    assert k >= 0
    return out[:k].tobytes()


def ref_index_stream(R, data: bytes, begin: int = 0, max_payload: int = DEFAULT_MAX_PAYLOAD):
    """The reference's receive loop (co_ws_server.c:107-169) around its own
    co_ws_frame_deserialize: (starts, consumed, stop)."""
    f = R.ref_index_stream
    f.argtypes = [_vp, C.c_ulonglong, C.c_ulonglong, C.c_ulonglong, _vp, C.c_ulonglong,
                  C.POINTER(C.c_ulonglong), C.POINTER(C.c_int)]
    f.restype = C.c_longlong
    src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    cap = len(data) // 2 + 1
    starts = np.zeros(cap, dtype=np.uint64)
    consumed, stop = C.c_ulonglong(), C.c_int()
    k = f(_ptr(src), len(data), begin, max_payload, _ptr(starts), cap, C.byref(consumed),
          C.byref(stop))
    return starts[:k], int(consumed.value), int(stop.value)


def ref_ws_accept_key(R, key: bytes) -> str:
    """The reference's co_sha1 + co_base64_encode on key || GUID."""
    f = R.ref_ws_accept_key
    f.argtypes = [C.c_char_p, C.c_ulonglong, C.c_char_p, C.c_ulonglong]
    f.restype = C.c_int
    out = C.create_string_buffer(64)
    assert f(key, len(key), out, 64) == 28
    return out.value.decode()


def ref_h2_recv(R, data: bytes, index: int = 0, S: int = 16384):
    f = R.ref_h2_recv
    f.argtypes = [_vp, C.c_ulonglong, C.POINTER(C.c_ulonglong), C.c_uint,
                  C.POINTER(C.c_uint), C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                  C.POINTER(C.c_uint), _vp, C.c_ulonglong, C.POINTER(C.c_ulonglong)]
    f.restype = C.c_int
    src = np.frombuffer(data, dtype=np.uint8)
    out = np.zeros(len(data) + 1, dtype=np.uint8)
    idx = C.c_ulonglong(index)
    ln, ty, fl, sid = C.c_uint(), C.c_uint(), C.c_uint(), C.c_uint()
    plen = C.c_ulonglong()
    r = f(_ptr(src), len(data), C.byref(idx), S, C.byref(ln), C.byref(ty), C.byref(fl),
          C.byref(sid), _ptr(out), out.size, C.byref(plen))
    return dict(rc=r, index=idx.value, length=ln.value, type=ty.value, flags=fl.value,
                sid=sid.value, payload=out[:plen.value].tobytes())
