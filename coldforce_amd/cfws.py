"""Python binding of libcfws.so (the MI355X WebSocket frame codec).

The product is the C ABI in ``include/cfws.h`` / ``include/cfws_co_ws_frame.h``;
this module only exposes it to the tests and ``bench.py`` through ctypes,
with torch supplying device memory and streams. It never falls back to a
CPU implementation: if the library or a gfx950 device is missing, calls
raise :class:`CodecError`.

Names mirror the reference: ``serialize`` = ``co_ws_frame_serialize``
(``src/ws/co_ws_frame.c:21-119``) over a batch, ``deserialize`` =
``co_ws_frame_deserialize`` (``co_ws_frame.c:121-247``) at each frame start.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CFWS_LIB") or os.path.join(HERE, "libcfws.so")   # CFWS_LIB: A/B builds

OK = 0
ERROR_INVALID_ARGUMENT, ERROR_WORKSPACE, ERROR_HIP, ERROR_NO_DEVICE = -1, -2, -3, -4   # cfws.h
PARSE_COMPLETE = 0
PARSE_MORE_DATA = 1
ERROR_INVALID_FRAME = -7001
ERROR_DATA_TOO_BIG = -7005
ERROR_OUT_OF_MEMORY = -7006
DEFAULT_MAX_PAYLOAD = 32 * 1024 * 1024          # co_ws_config.h:15
DESERIALIZE_REASSEMBLE = 1                      # include/cfws.h

OPCODE_CONTINUATION, OPCODE_TEXT, OPCODE_BINARY = 0x0, 0x1, 0x2
OPCODE_CLOSE, OPCODE_PING, OPCODE_PONG = 0x8, 0x9, 0xA

# cfws_frame_desc_t, 32 bytes.
DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("wire_off", "<u8"),
                       ("payload_size", "<u8"), ("mask_key", "<u4"),
                       ("fin", "u1"), ("opcode", "u1"), ("mask", "u1"),
                       ("header_size", "u1")])
assert DESC_DTYPE.itemsize == 32

# cfws_frame_info_t, 8 bytes (the compact output of the slot / scatter receives).
INFO_DTYPE = np.dtype([("payload_size", "<u4"), ("fin", "u1"), ("opcode", "u1"), ("status", "<i2")])
assert INFO_DTYPE.itemsize == 8

# Every function include/*.h declares (tests check the exports against the
# headers themselves).
BATCH_SYMBOLS = (
    "cfws_init", "cfws_init_device", "cfws_device_copy", "cfws_time_next_pass", "cfws_deserialize_pass_kernel", "cfws_serialize_uniform_pass_kernel", "cfws_deserialize_slots_pass_kernel", "cfws_bind_thread_device", "cfws_thread_device", "cfws_last_error", "cfws_version", "cfws_workspace_size",
    "cfws_serialize_plan", "cfws_serialize_execute", "cfws_serialize_batch", "cfws_serialize_uniform",
    "cfws_deserialize_plan", "cfws_deserialize_execute", "cfws_deserialize_batch",
    "cfws_deserialize_slots", "cfws_deserialize_scatter", "cfws_deserialize_slots_info",
    "cfws_deserialize_scatter_info", "cfws_deserialize_slots_uniform", "cfws_xor_mask", "cfws_draw_mask_keys", "cfws_draw_mask_keys_seeded",
    "cfws_release_thread_resources", "cfws_set_dropin_gpu_min", "cfws_dropin_gpu_min",
    "cfws_fill_splitmix", "cfws_pipeline_create", "cfws_pipeline_destroy",
    "cfws_pipeline_serialize", "cfws_pipeline_deserialize", "cfws_pipeline_receive",
    "cfws_h2_serialize_workspace_size", "cfws_h2_serialize_batch",
    "cfws_h2_deserialize_workspace_size", "cfws_h2_deserialize_batch",
    "cfws_index_frames", "cfws_index_workspace_size", "cfws_index_frames_batch",
    "cfws_ws_accept_keys_batch", "cfws_encode_headers", "cfws_parse_headers",
    "cfws_mask_batch", "cfws_mask_batch_packed", "cfws_unmask_batch", "cfws_copy_to_host",
    "cfws_mapped_device_pointer",
    "cfws_pipeline_set_d2h", "cfws_graph_serialize", "cfws_graph_deserialize", "cfws_graph_launch",
    "cfws_graph_destroy", "cfws_pipeline_h2_serialize", "cfws_pipeline_h2_deserialize",
)
DROPIN_SYMBOLS = (
    "co_ws_frame_serialize", "co_ws_frame_deserialize", "co_ws_frame_create",
    "co_ws_frame_destroy", "co_ws_frame_get_fin", "co_ws_frame_get_opcode",
    "co_ws_frame_get_payload_size", "co_ws_frame_get_payload_data",
    "co_ws_config_set_max_receive_payload_size", "co_ws_config_get_max_receive_payload_size",
)


class CodecError(RuntimeError):
    pass


class CoArray(C.Structure):
    """co_array_t / co_byte_array_t (inc/coldforce/core/co_array.h:16-23)."""
    _fields_ = [("capacity", C.c_size_t), ("count", C.c_size_t),
                ("element_size", C.c_size_t), ("buffer", C.c_void_p)]


class CoWsFrameHeader(C.Structure):
    _fields_ = [("fin", C.c_bool), ("opcode", C.c_uint8), ("payload_size", C.c_uint64)]


class CoWsFrame(C.Structure):
    """co_ws_frame_t (inc/coldforce/ws/co_ws_frame.h:36-49)."""
    _fields_ = [("header", CoWsFrameHeader), ("payload_data", C.c_void_p)]


_vp, _u64, _sz, _u32 = C.c_void_p, C.c_uint64, C.c_size_t, C.c_uint32
_lib = None


def lib(path: str = LIB_PATH) -> C.CDLL:
    """Load libcfws.so. torch is imported first so that the library binds to
    the HIP runtime torch already loaded (one runtime per process)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (HIP runtime first)
    if not os.path.exists(path):
        raise CodecError(f"{path} not built (run `make`); there is no CPU fallback")
    L = C.CDLL(path)
    sig = {
        "cfws_init": ([], C.c_int),
        "cfws_last_error": ([], C.c_char_p),
        "cfws_version": ([], C.c_char_p),
        "cfws_workspace_size": ([_sz, _u64], _sz),
        "cfws_serialize_plan": ([_vp, _sz, _u64, _vp, _vp, _sz, _vp], C.c_int),
        "cfws_serialize_execute": ([_vp, _vp, _sz, _vp, _u64, _vp, _vp], C.c_int),
        "cfws_serialize_batch": ([_vp, _vp, _sz, _vp, _u64, _vp, _vp, _sz, _vp], C.c_int),
        "cfws_serialize_uniform": ([_vp, _vp, _sz, _u64, C.c_uint8, C.c_uint8, C.c_uint8, _vp, _u64, _vp,
                                    _vp], C.c_int),
        "cfws_deserialize_plan": ([_vp, _u64, _vp, _sz, _u64, _u32, _u32, _vp, _vp, _u64, _vp,
                                   _vp, _sz, _vp], C.c_int),
        "cfws_deserialize_execute": ([_vp, _vp, _vp, _sz, _u32, _vp, _u64, _vp, _vp], C.c_int),
        "cfws_deserialize_batch": ([_vp, _u64, _vp, _sz, _u64, _u32, _u32, _vp, _vp, _vp, _u64,
                                    _vp, _vp, _sz, _vp], C.c_int),
        "cfws_deserialize_slots": ([_vp, _u64, _vp, _sz, _u64, _u64, _vp, _vp, _vp, _u64, _vp, _vp],
                                   C.c_int),
        "cfws_deserialize_scatter": ([_vp, _u64, _vp, _vp, _sz, _u64, _u64, _vp, _vp, _vp, _u64, _vp],
                                     C.c_int),
        "cfws_deserialize_slots_info": ([_vp, _u64, _vp, _sz, _u64, _u64, _vp, _vp, _u64, _vp, _vp], C.c_int),
        "cfws_deserialize_scatter_info": ([_vp, _u64, _vp, _vp, _sz, _u64, _u64, _vp, _vp, _u64, _vp],
                                          C.c_int),
        "cfws_deserialize_slots_uniform": ([_vp, _u64, _sz, _u64, _u64, _u64, _vp, _vp, _u64, _vp, _vp, _vp],
                                           C.c_int),
        "cfws_encode_headers": ([_vp, _sz, _vp, _u64, _vp], C.c_int),
        "cfws_parse_headers": ([_vp, _u64, _vp, _sz, _u64, _vp, _vp, _vp], C.c_int),
        "cfws_mask_batch": ([_vp, _vp, _sz, _u64, _vp, _u64, _vp], C.c_int),
        "cfws_mask_batch_packed": ([_vp, _vp, _sz, _u64, _vp, _u64, _vp], C.c_int),
        "cfws_unmask_batch": ([_vp, _vp, _vp, _sz, _u64, _vp, _u64, _vp], C.c_int),
        "cfws_copy_to_host": ([_vp, _vp, _u64, _vp], C.c_int),
        "cfws_pipeline_set_d2h": ([_vp, C.c_int], C.c_int),
        "cfws_graph_serialize": ([_vp, _vp, _sz, _vp, _u64, _vp, _vp, _sz, _vp], C.c_int),
        "cfws_graph_deserialize": ([_vp, _u64, _vp, _sz, _u64, _u32, _u32, _vp, _vp, _vp, _u64, _vp,
                                    _vp, _sz, _vp], C.c_int),
        "cfws_graph_launch": ([_vp, _vp], C.c_int),
        "cfws_pipeline_h2_serialize": ([_vp, _vp, _vp, _sz, _u32, _u32, _vp, _u64, _vp], C.c_int),
        "cfws_pipeline_h2_deserialize": ([_vp, _vp, _u64, _vp, _sz, _u32, _u64, _u32, _vp, _vp, _vp,
                                          _vp, _vp, _u64, _vp], C.c_int),
        "cfws_graph_destroy": ([_vp], None),
        "cfws_mapped_device_pointer": ([_vp], _vp),
        "cfws_xor_mask": ([_vp, _vp, _u64, _u32, _u32, _vp], C.c_int),
        "cfws_draw_mask_keys": ([_sz, _vp, _vp], None),
        "cfws_draw_mask_keys_seeded": ([_u32, _sz, _vp, _vp], C.c_int),
        "cfws_release_thread_resources": ([], None),
        "cfws_init_device": ([C.c_int], C.c_int),
        "cfws_device_copy": ([_vp, _vp, _u64, _vp], C.c_int),
        "cfws_time_next_pass": ([_vp, _vp], C.c_int),
        "cfws_deserialize_pass_kernel": ([_sz, _u64, _u32, _u32, _u64], C.c_char_p),
        "cfws_serialize_uniform_pass_kernel": ([_u64, C.c_uint8], C.c_char_p),
        "cfws_deserialize_slots_pass_kernel": ([_sz, _u64, _u64], C.c_char_p),
        "cfws_bind_thread_device": ([C.c_int], C.c_int),
        "cfws_thread_device": ([], C.c_int),
        "cfws_set_dropin_gpu_min": ([_sz], None),
        "cfws_dropin_gpu_min": ([], _sz),
        "cfws_fill_splitmix": ([_vp, _u64, _u64, _u64, _vp], C.c_int),
        "cfws_h2_serialize_workspace_size": ([_sz, _u64, _u64, _u32], _sz),
        "cfws_h2_serialize_batch": ([_vp, _vp, _sz, _u32, _u32, _vp, _u64, _vp, _u64, _vp, _vp,
                                     _sz, _vp], C.c_int),
        "cfws_h2_deserialize_workspace_size": ([_sz, _u64, _u64], _sz),
        "cfws_h2_deserialize_batch": ([_vp, _u64, _vp, _sz, _u32, _vp, _vp, _u64, _u64, _u32, _vp,
                                       _vp, _vp, _u64, _vp, C.POINTER(_sz), _vp, _sz, _vp],
                                      C.c_int),
        "cfws_index_frames": ([_vp, _u64, _u64, _u64, _vp, _sz, C.POINTER(_u64),
                               C.POINTER(C.c_int32)], _sz),
        "cfws_index_workspace_size": ([_sz], _sz),
        "cfws_index_frames_batch": ([_vp, _vp, _vp, _sz, _u64, _vp, _u64, _vp, _vp, _vp, _vp, _vp,
                                     _sz, _vp], C.c_int),
        "cfws_ws_accept_keys_batch": ([_vp, _vp, _sz, _vp, _vp], C.c_int),
        "cfws_pipeline_create": ([_u64, _sz, C.c_int, C.POINTER(_vp)], C.c_int),
        "cfws_pipeline_destroy": ([_vp], None),
        "cfws_pipeline_serialize": ([_vp, _vp, _vp, _sz, _vp, _u64, C.POINTER(_u64)], C.c_int),
        "cfws_pipeline_deserialize": ([_vp, _vp, _u64, _vp, _sz, _u64, _u32, _u32, _vp, _vp, _vp,
                                       _u64, C.POINTER(_u64)], C.c_int),
        "cfws_pipeline_receive": ([_vp, _vp, _u64, _u64, _u64, _u32, _vp, _vp, C.POINTER(_sz),
                                   C.POINTER(_u64), C.POINTER(C.c_int32), _vp, _u64,
                                   C.POINTER(_u64)], C.c_int),
        "co_ws_frame_serialize": ([C.c_bool, C.c_uint8, C.c_bool, _vp, _sz, C.POINTER(CoArray)],
                                  C.c_bool),
        "co_ws_frame_deserialize": ([C.POINTER(CoWsFrame), _vp, _sz, C.POINTER(C.c_size_t)],
                                    C.c_int),
        "co_ws_frame_create": ([], C.POINTER(CoWsFrame)),
        "co_ws_frame_destroy": ([C.POINTER(CoWsFrame)], None),
        "co_ws_frame_get_fin": ([C.POINTER(CoWsFrame)], C.c_bool),
        "co_ws_frame_get_opcode": ([C.POINTER(CoWsFrame)], C.c_uint8),
        "co_ws_frame_get_payload_size": ([C.POINTER(CoWsFrame)], C.c_uint64),
        "co_ws_frame_get_payload_data": ([C.POINTER(CoWsFrame)], _vp),
        "co_ws_config_set_max_receive_payload_size": ([_sz], None),
        "co_ws_config_get_max_receive_payload_size": ([], _sz),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise CodecError(f"{what} failed rc={rc}: {lib().cfws_last_error().decode()}")


def init() -> None:
    """Raise unless a gfx950 device is usable (no CPU fallback exists)."""
    _check(lib().cfws_init(), "cfws_init")


def _p(t) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(stream) -> int | None:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


# ---- host helpers ----------------------------------------------------------

def draw_mask_keys(n: int, mask_flags=None, seed: int | None = None) -> np.ndarray:
    """Keys exactly as n sequential co_ws_frame_serialize calls draw them:
    from the process's random() state, or, with a seed, as they would right
    after srandom(seed) (cfws_draw_mask_keys_seeded: a private copy of the
    generator, which no other thread's rand() can disturb; the HIP and torch
    runtimes' libraries call rand()/random() on threads of their own)."""
    keys = np.zeros(n, dtype=np.uint32)
    mf = None if mask_flags is None else np.ascontiguousarray(mask_flags, dtype=np.uint8)
    mp = None if mf is None else mf.ctypes.data
    if seed is None:
        lib().cfws_draw_mask_keys(n, mp, keys.ctypes.data)
    else:
        _check(lib().cfws_draw_mask_keys_seeded(seed, n, mp, keys.ctypes.data),
               "cfws_draw_mask_keys_seeded")
    return keys


def header_sizes(sizes: np.ndarray, masks: np.ndarray) -> np.ndarray:
    sizes = np.asarray(sizes, dtype=np.uint64)
    ext = np.where(sizes > 65535, 8, np.where(sizes > 125, 2, 0))
    return (2 + ext + 4 * (np.asarray(masks) != 0)).astype(np.uint64)


def desc_to_device(desc: np.ndarray, device="cuda"):
    import torch
    raw = np.ascontiguousarray(desc, dtype=DESC_DTYPE).view(np.uint8).reshape(-1, 32)
    return torch.from_numpy(raw.copy()).to(device)


def desc_from_device(t) -> np.ndarray:
    return t.cpu().numpy().reshape(-1).view(DESC_DTYPE).copy()


def workspace(n_frames: int, out_capacity: int, device="cuda"):
    import torch
    nbytes = lib().cfws_workspace_size(n_frames, out_capacity)
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


# ---- batch API ---------------------------------------------------------------

def serialize_plan(desc_t, wire_capacity: int, total_t, ws_t, stream=None) -> None:
    _check(lib().cfws_serialize_plan(_p(desc_t), desc_t.shape[0], wire_capacity, _p(total_t),
                                     _p(ws_t), ws_t.numel(), _stream(stream)),
           "cfws_serialize_plan")


def serialize_execute(payload_t, desc_t, wire_t, ws_t, wire_capacity: int | None = None,
                      stream=None) -> None:
    cap = wire_t.numel() if wire_capacity is None else wire_capacity
    _check(lib().cfws_serialize_execute(_p(payload_t), _p(desc_t), desc_t.shape[0], _p(wire_t),
                                        cap, _p(ws_t), _stream(stream)),
           "cfws_serialize_execute")


def serialize(payload_t, desc_t, wire_t, ws_t=None, total_t=None, stream=None):
    """Serialize every frame of desc_t into wire_t; returns the total tensor."""
    import torch
    n = desc_t.shape[0]
    if ws_t is None:
        ws_t = workspace(n, wire_t.numel(), wire_t.device)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=wire_t.device)
    _check(lib().cfws_serialize_batch(_p(payload_t), _p(desc_t), n, _p(wire_t), wire_t.numel(),
                                      _p(total_t), _p(ws_t), ws_t.numel(), _stream(stream)),
           "cfws_serialize_batch")
    return total_t


def uniform_frame_bytes(payload_size: int, mask: bool) -> int:
    """W: wire bytes of one frame of a uniform batch (header + payload)."""
    return int(header_sizes(np.array([payload_size]), np.array([mask]))[0]) + payload_size


def serialize_uniform(payload_t, keys_t, n: int, payload_size: int, wire_t, fin: bool = True,
                      opcode: int = OPCODE_BINARY, mask: bool = True, total_t=None,
                      wire_capacity: int | None = None, stream=None):
    """cfws_serialize_uniform: n frames of payload_size bytes each, frame i's
    payload at payload_t[i * payload_size:], its key keys_t[i] (uint32 /
    int32 tensor; None when unmasked). Returns total_t (n * W) or None."""
    cap = wire_t.numel() if wire_capacity is None else wire_capacity
    _check(lib().cfws_serialize_uniform(_p(payload_t), _p(keys_t), n, payload_size, int(bool(fin)), opcode,
                                        int(bool(mask)), _p(wire_t), cap, _p(total_t), _stream(stream)),
           "cfws_serialize_uniform")
    return total_t


def deserialize_plan(wire_t, wire_size: int, index_t, desc_t, status_t, payload_capacity: int,
                     total_t, ws_t, max_payload: int = DEFAULT_MAX_PAYLOAD, align: int = 16,
                     flags: int = 0, stream=None) -> None:
    _check(lib().cfws_deserialize_plan(_p(wire_t), wire_size, _p(index_t), index_t.numel(),
                                       max_payload, align, flags, _p(desc_t), _p(status_t),
                                       payload_capacity, _p(total_t), _p(ws_t), ws_t.numel(),
                                       _stream(stream)),
           "cfws_deserialize_plan")


def deserialize_execute(wire_t, desc_t, status_t, payload_t, ws_t,
                        payload_capacity: int | None = None, flags: int = 0,
                        stream=None) -> None:
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_execute(_p(wire_t), _p(desc_t), _p(status_t), desc_t.shape[0],
                                          flags, _p(payload_t), cap, _p(ws_t), _stream(stream)),
           "cfws_deserialize_execute")


def deserialize(wire_t, wire_size: int, index_t, payload_t, desc_t=None, status_t=None,
                ws_t=None, total_t=None, max_payload: int = DEFAULT_MAX_PAYLOAD,
                align: int = 16, flags: int = 0, stream=None):
    """Deserialize the frame starting at each index_t[i] of wire_t[:wire_size].
    Returns (desc_t, status_t, total_t)."""
    import torch
    n = index_t.numel()
    dev = wire_t.device
    if desc_t is None:
        desc_t = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    if status_t is None:
        status_t = torch.empty(n, dtype=torch.int32, device=dev)
    if ws_t is None:
        ws_t = workspace(n, payload_t.numel(), dev)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=dev)
    _check(lib().cfws_deserialize_batch(_p(wire_t), wire_size, _p(index_t), n, max_payload, align,
                                        flags, _p(desc_t), _p(status_t), _p(payload_t),
                                        payload_t.numel(), _p(total_t), _p(ws_t), ws_t.numel(),
                                        _stream(stream)),
           "cfws_deserialize_batch")
    return desc_t, status_t, total_t


def deserialize_slots(wire_t, wire_size: int, index_t, payload_t, slot_bytes: int, desc_t=None,
                      status_t=None, total_t=None, max_payload: int = DEFAULT_MAX_PAYLOAD,
                      payload_capacity: int | None = None, stream=None):
    """cfws_deserialize_slots: frame i's payload at i * slot_bytes of payload_t.
    Returns (desc_t, status_t, total_t)."""
    import torch
    n = index_t.numel()
    dev = wire_t.device
    if desc_t is None:
        desc_t = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    if status_t is None:
        status_t = torch.empty(n, dtype=torch.int32, device=dev)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=dev)
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_slots(_p(wire_t), wire_size, _p(index_t), n, max_payload, slot_bytes,
                                        _p(desc_t), _p(status_t), _p(payload_t), cap, _p(total_t),
                                        _stream(stream)),
           "cfws_deserialize_slots")
    return desc_t, status_t, total_t


def deserialize_scatter(wire_t, wire_size: int, index_t, payload_off_t, payload_t, max_slot: int,
                        desc_t=None, status_t=None, max_payload: int = DEFAULT_MAX_PAYLOAD,
                        payload_capacity: int | None = None, stream=None):
    """cfws_deserialize_scatter: frame i's payload at payload_off_t[i] of
    payload_t. Returns (desc_t, status_t)."""
    import torch
    n = index_t.numel()
    dev = wire_t.device
    if desc_t is None:
        desc_t = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    if status_t is None:
        status_t = torch.empty(n, dtype=torch.int32, device=dev)
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_scatter(_p(wire_t), wire_size, _p(index_t), _p(payload_off_t), n, max_payload,
                                          max_slot, _p(desc_t), _p(status_t), _p(payload_t), cap,
                                          _stream(stream)),
           "cfws_deserialize_scatter")
    return desc_t, status_t


def deserialize_slots_info(wire_t, wire_size: int, index_t, payload_t, slot_bytes: int, info_t=None,
                           total_t=None, max_payload: int = DEFAULT_MAX_PAYLOAD,
                           payload_capacity: int | None = None, stream=None):
    """cfws_deserialize_slots_info: the slot receive writing one 8-byte
    cfws_frame_info_t per frame (info_t: (n, 8) uint8). Returns (info_t, total_t)."""
    import torch
    n = index_t.numel()
    dev = wire_t.device
    if info_t is None:
        info_t = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=dev)
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_slots_info(_p(wire_t), wire_size, _p(index_t), n, max_payload, slot_bytes,
                                             _p(info_t), _p(payload_t), cap, _p(total_t), _stream(stream)),
           "cfws_deserialize_slots_info")
    return info_t, total_t


def deserialize_scatter_info(wire_t, wire_size: int, index_t, payload_off_t, payload_t, max_slot: int,
                             info_t=None, max_payload: int = DEFAULT_MAX_PAYLOAD,
                             payload_capacity: int | None = None, stream=None):
    """cfws_deserialize_scatter_info. Returns info_t ((n, 8) uint8)."""
    import torch
    n = index_t.numel()
    if info_t is None:
        info_t = torch.empty((n, 8), dtype=torch.uint8, device=wire_t.device)
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_scatter_info(_p(wire_t), wire_size, _p(index_t), _p(payload_off_t), n,
                                               max_payload, max_slot, _p(info_t), _p(payload_t), cap,
                                               _stream(stream)),
           "cfws_deserialize_scatter_info")
    return info_t


def deserialize_slots_uniform(wire_t, wire_size: int, n: int, frame_stride: int, payload_t, slot_bytes: int,
                              info_t=None, total_t=None, mismatch_t=None,
                              max_payload: int = DEFAULT_MAX_PAYLOAD, payload_capacity: int | None = None,
                              stream=None):
    """cfws_deserialize_slots_uniform: the info slot receive with frame i at
    i * frame_stride of the wire (no index). mismatch_t (one int32, may be
    None): the frames that are not COMPLETE frames of frame_stride bytes.
    Returns (info_t, total_t)."""
    import torch
    dev = wire_t.device
    if info_t is None:
        info_t = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=dev)
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_deserialize_slots_uniform(_p(wire_t), wire_size, n, frame_stride, max_payload, slot_bytes,
                                                _p(info_t), _p(payload_t), cap, _p(total_t), _p(mismatch_t),
                                                _stream(stream)),
           "cfws_deserialize_slots_uniform")
    return info_t, total_t


def info_from_device(t) -> np.ndarray:
    return t.cpu().numpy().reshape(-1).view(INFO_DTYPE).copy()


# ---- HIP graphs of a batch (cfws_graph_*) -----------------------------------

class Graph:
    """One captured cfws_serialize_batch / cfws_deserialize_batch over fixed
    arenas (the tensors must outlive the graph); launch() replays it."""

    def __init__(self, h):
        self.h = h

    @classmethod
    def serialize(cls, payload_t, desc_t, wire_t, ws_t, total_t):
        h = _vp()
        _check(lib().cfws_graph_serialize(_p(payload_t), _p(desc_t), desc_t.shape[0], _p(wire_t),
                                          wire_t.numel(), _p(total_t), _p(ws_t), ws_t.numel(),
                                          C.byref(h)), "cfws_graph_serialize")
        return cls(h)

    @classmethod
    def deserialize(cls, wire_t, wire_size: int, index_t, desc_t, status_t, payload_t, ws_t, total_t,
                    max_payload: int = DEFAULT_MAX_PAYLOAD, align: int = 16, flags: int = 0):
        h = _vp()
        _check(lib().cfws_graph_deserialize(_p(wire_t), wire_size, _p(index_t), index_t.numel(),
                                            max_payload, align, flags, _p(desc_t), _p(status_t),
                                            _p(payload_t), payload_t.numel(), _p(total_t), _p(ws_t),
                                            ws_t.numel(), C.byref(h)), "cfws_graph_deserialize")
        return cls(h)

    def launch(self, stream=None) -> None:
        _check(lib().cfws_graph_launch(self.h, _stream(stream)), "cfws_graph_launch")

    def close(self):
        if self.h:
            lib().cfws_graph_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- host memory ---------------------------------------------------------------

_hiprt = None


def _hip():
    global _hiprt
    if _hiprt is None:
        lib()                                          # the HIP runtime torch loaded
        h = C.CDLL("libamdhip64.so")
        h.hipHostMalloc.argtypes = [C.POINTER(_vp), _sz, C.c_uint]
        h.hipHostMalloc.restype = C.c_int
        h.hipHostFree.argtypes = [_vp]
        h.hipHostFree.restype = C.c_int
        _hiprt = h
    return _hiprt


HIP_HOST_MALLOC_MAPPED = 0x2
HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000


class TimingEvent:
    """A HIP timing event recorded on torch's current stream (or `stream`),
    created with hipEventDisableSystemFence: recording it adds no
    system-scope fence (cache writeback + invalidate) to the stream. Four
    torch.cuda.Event records per config-2 step left ~6 us of idle GPU at
    each one, 0.5 % of the step; these leave none, and time the same
    (tools/event_gap_probe.py). Same calls as torch.cuda.Event: record(),
    elapsed_time(end) in ms (after a synchronize)."""

    def __init__(self):
        h = _hip()
        if not hasattr(h, "_cfws_event_sigs"):
            h.hipEventCreateWithFlags.argtypes = [C.POINTER(_vp), C.c_uint]
            h.hipEventRecord.argtypes = [_vp, _vp]
            h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), _vp, _vp]
            h.hipEventDestroy.argtypes = [_vp]
            h._cfws_event_sigs = True
        self._h = h
        self.ev = _vp()
        rc = h.hipEventCreateWithFlags(C.byref(self.ev), HIP_EVENT_DISABLE_SYSTEM_FENCE)
        if rc != 0:
            raise CodecError(f"hipEventCreateWithFlags rc={rc}")

    def record(self, stream=None) -> None:
        rc = self._h.hipEventRecord(self.ev, _vp(_stream(stream)))
        if rc != 0:
            raise CodecError(f"hipEventRecord rc={rc}")

    def elapsed_time(self, end: "TimingEvent") -> float:
        ms = C.c_float()
        rc = self._h.hipEventElapsedTime(C.byref(ms), self.ev, end.ev)
        if rc != 0:
            # the failure also sets the thread's last HIP error: clear it, or
            # the next library call's launch check reports it as its own
            self._h.hipGetLastError()
            raise CodecError(f"hipEventElapsedTime rc={rc}")
        return ms.value

    def __del__(self):
        if getattr(self, "ev", None) and self.ev.value:
            self._h.hipEventDestroy(self.ev)
            self.ev = _vp()


def mapped_host(nbytes: int):
    """A uint8 torch tensor over pinned host memory allocated MAPPED
    (hipHostMalloc(..., hipHostMallocMapped)): the host pipeline writes such
    buffers with a kernel instead of an SDMA copy (cfws_copy_to_host). The
    memory is freed with the tensor."""
    import weakref

    import numpy as np
    import torch
    n = max(int(nbytes), 16)
    ptr = _vp()
    rc = _hip().hipHostMalloc(C.byref(ptr), n, HIP_HOST_MALLOC_MAPPED)
    if rc != 0 or not ptr.value:
        raise CodecError(f"hipHostMalloc({n}) failed rc={rc}")
    buf = (C.c_uint8 * n).from_address(ptr.value)
    weakref.finalize(buf, _hip().hipHostFree, ptr.value)
    return torch.from_numpy(np.ctypeslib.as_array(buf))


def copy_to_host(src_t, h_dst_ptr: int, n: int, stream=None) -> None:
    """Device -> mapped host copy by a kernel (cfws_copy_to_host)."""
    _check(lib().cfws_copy_to_host(_p(src_t), h_dst_ptr, n, _stream(stream)), "cfws_copy_to_host")


# ---- split ops (headers and payload XOR as separate passes) -----------------

def encode_headers(desc_t, wire_t, wire_capacity: int | None = None, stream=None) -> None:
    cap = wire_t.numel() if wire_capacity is None else wire_capacity
    _check(lib().cfws_encode_headers(_p(desc_t), desc_t.shape[0], _p(wire_t), cap,
                                     _stream(stream)), "cfws_encode_headers")


def parse_headers(wire_t, wire_size: int, index_t, desc_t, status_t,
                  max_payload: int = DEFAULT_MAX_PAYLOAD, stream=None) -> None:
    _check(lib().cfws_parse_headers(_p(wire_t), wire_size, _p(index_t), index_t.numel(),
                                    max_payload, _p(desc_t), _p(status_t), _stream(stream)),
           "cfws_parse_headers")


def mask_batch(payload_t, desc_t, wire_t, max_payload_size: int, wire_capacity: int | None = None,
               stream=None, packed: bool = False) -> None:
    """cfws_mask_batch, or with packed=True cfws_mask_batch_packed (frames
    back to back, headers as cfws_encode_headers writes them)."""
    cap = wire_t.numel() if wire_capacity is None else wire_capacity
    fn = lib().cfws_mask_batch_packed if packed else lib().cfws_mask_batch
    _check(fn(_p(payload_t), _p(desc_t), desc_t.shape[0], max_payload_size, _p(wire_t), cap,
              _stream(stream)), "cfws_mask_batch")


def unmask_batch(wire_t, desc_t, status_t, payload_t, max_payload_size: int,
                 payload_capacity: int | None = None, stream=None) -> None:
    cap = payload_t.numel() if payload_capacity is None else payload_capacity
    _check(lib().cfws_unmask_batch(_p(wire_t), _p(desc_t), _p(status_t), desc_t.shape[0],
                                   max_payload_size, _p(payload_t), cap, _stream(stream)),
           "cfws_unmask_batch")


def xor_mask(src_t, dst_t, n: int, key: int, phase: int = 0, stream=None) -> None:
    _check(lib().cfws_xor_mask(_p(src_t), _p(dst_t), n, key, phase, _stream(stream)),
           "cfws_xor_mask")


def time_next_pass(start: "TimingEvent | None", stop: "TimingEvent | None") -> None:
    """cfws_time_next_pass: the calling thread's next streaming pass records
    start before and stop after its launch (None, None clears)."""
    _check(lib().cfws_time_next_pass(start.ev if start else None, stop.ev if stop else None),
           "cfws_time_next_pass")


def device_copy(src_t, dst_t, n: int | None = None, stream=None) -> None:
    """cfws_device_copy: dst_t[:n] = src_t[:n] (n a multiple of 16)."""
    n = src_t.numel() if n is None else n
    _check(lib().cfws_device_copy(_p(src_t), _p(dst_t), n, _stream(stream)), "cfws_device_copy")


def fill_splitmix(dst_t, seed: int, byte_base: int = 0, n: int | None = None, stream=None) -> None:
    n = dst_t.numel() if n is None else n
    _check(lib().cfws_fill_splitmix(_p(dst_t), n, seed, byte_base, _stream(stream)),
           "cfws_fill_splitmix")


# ---- drop-in per-frame API (co_ws_frame_*) ---------------------------------

_libc = None


def _c():
    global _libc
    if _libc is None:
        _libc = C.CDLL(None)
        _libc.malloc.restype = C.c_void_p
        _libc.malloc.argtypes = [C.c_size_t]
        _libc.free.argtypes = [C.c_void_p]
    return _libc


def byte_array_create() -> CoArray:
    """co_byte_array_create(): capacity 8, element_size 1 (co_array.c:15-40)."""
    a = CoArray()
    a.capacity, a.count, a.element_size = 8, 0, 1
    a.buffer = _c().malloc(8)
    return a


def byte_array_bytes(a: CoArray) -> bytes:
    return C.string_at(a.buffer, a.count) if a.count else b""


def byte_array_destroy(a: CoArray) -> None:
    _c().free(a.buffer)
    a.buffer = None


def frame_serialize(fin: bool, opcode: int, mask: bool, data: bytes, buf: CoArray | None = None):
    """co_ws_frame_serialize through the drop-in; returns (ok, wire bytes)."""
    own = buf is None
    if own:
        buf = byte_array_create()
    src = C.create_string_buffer(data, len(data)) if data else None
    ok = lib().co_ws_frame_serialize(fin, opcode, mask, src, len(data), C.byref(buf))
    out = byte_array_bytes(buf)
    if own:
        byte_array_destroy(buf)
    return ok, out


def frame_deserialize(data: bytes, index: int = 0):
    """co_ws_frame_deserialize through the drop-in on a fresh frame.
    Returns dict(rc, index, fin, opcode, payload_size, payload|None), the
    payload including its NUL terminator, like oracle.ref_deserialize."""
    L = lib()
    f = L.co_ws_frame_create()
    src = C.create_string_buffer(data, len(data))
    idx = C.c_size_t(index)
    rc = L.co_ws_frame_deserialize(f, src, len(data), C.byref(idx))
    fr = f.contents
    payload = None
    if rc == 0 and fr.payload_data:
        payload = C.string_at(fr.payload_data, fr.header.payload_size + 1)
    out = dict(rc=rc, index=idx.value, fin=bool(fr.header.fin), opcode=fr.header.opcode,
               payload_size=fr.header.payload_size, payload=payload)
    L.co_ws_frame_destroy(f)
    return out


# ---- WebSocket over HTTP/2 ---------------------------------------------------

H2_DEFAULT_MAX_FRAME_SIZE = 16384
H2_PARSE_COMPLETE, H2_PARSE_MORE_DATA, H2_PARSE_ERROR, H2_NOT_DATA = 0, 1, -1, 3


def h2_wrapped_bound(wire_capacity: int, n_frames: int, S: int = H2_DEFAULT_MAX_FRAME_SIZE) -> int:
    return wire_capacity + 9 * (n_frames + wire_capacity // S + 1)


def h2_serialize(payload_t, desc_t, wire_t, h2_t, sid: int = 1, S: int = H2_DEFAULT_MAX_FRAME_SIZE,
                 ws_t=None, total_t=None, stream=None):
    """WS frames -> HTTP/2 DATA frames (co_http2_stream_send_ws_frame over a
    batch). wire_t is scratch for the WS wire bytes. Returns total_t."""
    import torch
    n = desc_t.shape[0]
    if ws_t is None:
        ws_t = torch.empty(lib().cfws_h2_serialize_workspace_size(n, wire_t.numel(), h2_t.numel(), S),
                           dtype=torch.uint8, device=h2_t.device)
    if total_t is None:
        total_t = torch.zeros(1, dtype=torch.int64, device=h2_t.device)
    _check(lib().cfws_h2_serialize_batch(_p(payload_t), _p(desc_t), n, sid, S, _p(wire_t),
                                         wire_t.numel(), _p(h2_t), h2_t.numel(), _p(total_t),
                                         _p(ws_t), ws_t.numel(), _stream(stream)),
           "cfws_h2_serialize_batch")
    return total_t


def h2_deserialize(h2_t, h2_size: int, index_t, pool_t, payload_t, S: int = H2_DEFAULT_MAX_FRAME_SIZE,
                   max_payload: int = DEFAULT_MAX_PAYLOAD, align: int = 16, ws_t=None, stream=None,
                   all_rows: bool = False):
    """HTTP/2 DATA frames at index_t -> pooled WS messages -> payloads.
    Returns (h2_status_t, msg_desc_t, msg_status_t, total_t, n_messages).
    n_messages is final on return; the tensors are written by work still
    queued on `stream` (synchronise it before reading them on another).
    all_rows: return every message row (one per DATA frame; rows past
    n_messages are empty entries) instead of the first n_messages."""
    import torch
    n = index_t.numel()
    dev = h2_t.device
    h2_status = torch.empty(n, dtype=torch.int32, device=dev)
    msg_desc = torch.empty((max(n, 1), 32), dtype=torch.uint8, device=dev)
    msg_status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)      # always written by the library
    if ws_t is None:
        ws_t = torch.empty(lib().cfws_h2_deserialize_workspace_size(n, pool_t.numel(), payload_t.numel()),
                           dtype=torch.uint8, device=dev)
    n_msg = C.c_size_t(0)
    _check(lib().cfws_h2_deserialize_batch(_p(h2_t), h2_size, _p(index_t), n, S, _p(h2_status),
                                           _p(pool_t), pool_t.numel(), max_payload, align,
                                           _p(msg_desc), _p(msg_status), _p(payload_t),
                                           payload_t.numel(), _p(total), C.byref(n_msg), _p(ws_t),
                                           ws_t.numel(), _stream(stream)),
           "cfws_h2_deserialize_batch")
    m = n_msg.value
    if all_rows:
        return h2_status, msg_desc, msg_status, total, m
    return h2_status, msg_desc[:m], msg_status[:m], total, m


# ---- receive-buffer frame indexing -----------------------------------------
INDEX_FULL = 2


def index_frames(buf: np.ndarray, begin: int = 0, end: int | None = None,
                 max_payload: int = DEFAULT_MAX_PAYLOAD, max_starts: int | None = None):
    """Host receive-loop walk of one connection's bytes buf[begin, end)
    (cfws_index_frames): (starts, consumed, stop)."""
    end = buf.size if end is None else end
    cap = max((end - begin) // 2 + 1, 1) if max_starts is None else max_starts
    starts = np.zeros(max(cap, 1), dtype=np.uint64)
    b = buf if buf.size else np.zeros(1, np.uint8)
    consumed, stop = _u64(0), C.c_int32(0)
    k = lib().cfws_index_frames(b.ctypes.data, begin, end, max_payload, starts.ctypes.data, cap,
                                C.byref(consumed), C.byref(stop))
    return starts[:k], int(consumed.value), int(stop.value)


def index_frames_batch(buf_t, begin_t, end_t, max_payload: int = DEFAULT_MAX_PAYLOAD,
                       starts_t=None, ws_t=None, stream=None):
    """Device receive-loop walk of many connections at once
    (cfws_index_frames_batch). Returns (starts_t, first_t, consumed_t,
    stop_t, total) -- total synchronises."""
    import torch
    n = begin_t.numel()
    dev = buf_t.device
    if starts_t is None:
        span = int((end_t - begin_t).clamp(min=0).sum().item()) if n else 0
        starts_t = torch.empty(max(span // 2 + n, 1), dtype=torch.int64, device=dev)
    first = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    consumed = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    stop = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    if ws_t is None:
        ws_t = torch.empty(lib().cfws_index_workspace_size(n), dtype=torch.uint8, device=dev)
    _check(lib().cfws_index_frames_batch(_p(buf_t), _p(begin_t), _p(end_t), n, max_payload,
                                         _p(starts_t), starts_t.numel(), _p(first), _p(consumed),
                                         _p(stop), _p(total), _p(ws_t), ws_t.numel(),
                                         _stream(stream)),
           "cfws_index_frames_batch")
    return starts_t, first[:n], consumed[:n], stop[:n], int(total.item())


# ---- handshake accept keys ---------------------------------------------------
WS_ACCEPT_SLOT = 32


def ws_accept_keys(keys, device="cuda", stream=None) -> list[str]:
    """Sec-WebSocket-Accept of every key (bytes) through
    cfws_ws_accept_keys_batch."""
    import torch
    off = np.zeros(len(keys) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(k) for k in keys])
    raw = np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy()
    d_keys = torch.from_numpy(raw).to(device)
    d_off = torch.from_numpy(off).to(device)
    out = torch.zeros(max(len(keys), 1) * WS_ACCEPT_SLOT, dtype=torch.uint8, device=device)
    _check(lib().cfws_ws_accept_keys_batch(_p(d_keys), _p(d_off), len(keys), _p(out),
                                           _stream(stream)), "cfws_ws_accept_keys_batch")
    h = out.cpu().numpy().reshape(-1, WS_ACCEPT_SLOT)
    return [bytes(h[i, :28]).decode() for i in range(len(keys))]


# ---- host-memory pipeline --------------------------------------------------

PIPELINE_D2H = {"auto": 0, "dma": 1, "kernel": 2}     # CFWS_PIPELINE_D2H_*


class Pipeline:
    """cfws_pipeline_*: the codec over host buffers (pinned numpy/torch
    memory recommended), H2D / kernels / D2H overlapped across `depth` slots."""

    def __init__(self, chunk_bytes: int = 64 << 20, max_frames: int = 1 << 18, depth: int = 3,
                 d2h: str | None = None):
        h = C.c_void_p()
        _check(lib().cfws_pipeline_create(chunk_bytes, max_frames, depth, C.byref(h)),
               "cfws_pipeline_create")
        self.h = h
        if d2h is not None:
            self.set_d2h(d2h)

    def set_d2h(self, mode: str) -> None:
        """'auto' | 'dma' | 'kernel': cfws_pipeline_set_d2h."""
        _check(lib().cfws_pipeline_set_d2h(self.h, PIPELINE_D2H[mode]), "cfws_pipeline_set_d2h")

    def close(self):
        if self.h:
            lib().cfws_pipeline_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def serialize(self, payload_ptr: int, desc: np.ndarray, wire_ptr: int, wire_capacity: int) -> int:
        """desc: host DESC_DTYPE array (wire_off/header_size filled in place)."""
        tot = C.c_uint64()
        _check(lib().cfws_pipeline_serialize(self.h, payload_ptr, desc.ctypes.data, len(desc),
                                             wire_ptr, wire_capacity, C.byref(tot)),
               "cfws_pipeline_serialize")
        return tot.value

    def deserialize(self, wire_ptr: int, wire_size: int, index: np.ndarray, payload_ptr: int,
                    payload_capacity: int, align: int = 16, max_payload: int = DEFAULT_MAX_PAYLOAD):
        """Returns (desc, status, total)."""
        index = np.ascontiguousarray(index, dtype=np.uint64)
        desc = np.zeros(len(index), dtype=DESC_DTYPE)
        status = np.zeros(len(index), dtype=np.int32)
        tot = C.c_uint64()
        _check(lib().cfws_pipeline_deserialize(self.h, wire_ptr, wire_size, index.ctypes.data,
                                               len(index), max_payload, align, 0,
                                               desc.ctypes.data, status.ctypes.data, payload_ptr,
                                               payload_capacity, C.byref(tot)),
               "cfws_pipeline_deserialize")
        return desc, status, tot.value

    def h2_serialize(self, payload_ptr: int, desc: np.ndarray, h2_ptr: int, h2_capacity: int,
                     sid: int = 1, S: int = H2_DEFAULT_MAX_FRAME_SIZE) -> int:
        """WS frames -> HTTP/2 DATA stream, host to host (cfws_pipeline_h2_serialize).
        desc: host DESC_DTYPE array (wire_off/header_size filled in place)."""
        tot = C.c_uint64()
        _check(lib().cfws_pipeline_h2_serialize(self.h, payload_ptr, desc.ctypes.data, len(desc), sid, S,
                                                h2_ptr, h2_capacity, C.byref(tot)),
               "cfws_pipeline_h2_serialize")
        return tot.value

    def h2_deserialize(self, h2_ptr: int, h2_size: int, index: np.ndarray, payload_ptr: int,
                       payload_capacity: int, S: int = H2_DEFAULT_MAX_FRAME_SIZE, align: int = 16,
                       max_payload: int = DEFAULT_MAX_PAYLOAD):
        """DATA frames at index -> messages -> payloads, host to host
        (cfws_pipeline_h2_deserialize). Returns (h2_status, msg_desc,
        msg_status, total)."""
        idx = np.ascontiguousarray(index, dtype=np.uint64)
        n = len(idx)
        h2_status = np.zeros(max(n, 1), dtype=np.int32)
        mdesc = np.zeros(max(n, 1), dtype=DESC_DTYPE)
        mstatus = np.zeros(max(n, 1), dtype=np.int32)
        nm, tot = C.c_size_t(0), C.c_uint64()
        _check(lib().cfws_pipeline_h2_deserialize(self.h, h2_ptr, h2_size, idx.ctypes.data, n, S,
                                                  max_payload, align, h2_status.ctypes.data,
                                                  mdesc.ctypes.data, mstatus.ctypes.data, C.byref(nm),
                                                  payload_ptr, payload_capacity, C.byref(tot)),
               "cfws_pipeline_h2_deserialize")
        m = nm.value
        return h2_status[:n], mdesc[:m], mstatus[:m], tot.value

    def receive(self, wire_ptr: int, begin: int, end: int, payload_ptr: int, payload_capacity: int,
                max_frames: int, align: int = 16, max_payload: int = DEFAULT_MAX_PAYLOAD):
        """The receive loop over host bytes [begin, end): index + deserialize.
        Returns (desc, status, consumed, stop, total)."""
        desc = np.zeros(max(max_frames, 1), dtype=DESC_DTYPE)
        status = np.zeros(max(max_frames, 1), dtype=np.int32)
        n = C.c_size_t(max_frames)
        consumed, stop, tot = C.c_uint64(), C.c_int32(), C.c_uint64()
        _check(lib().cfws_pipeline_receive(self.h, wire_ptr, begin, end, max_payload, align,
                                           desc.ctypes.data, status.ctypes.data, C.byref(n),
                                           C.byref(consumed), C.byref(stop), payload_ptr,
                                           payload_capacity, C.byref(tot)),
               "cfws_pipeline_receive")
        k = n.value
        return desc[:k], status[:k], consumed.value, stop.value, tot.value
