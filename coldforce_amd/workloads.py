"""Synthetic frame batches for the BASELINE.json configurations.

Each builder returns host-side descriptors (numpy, DESC_DTYPE); payload bytes
are generated on the device by ``cfws.fill_splitmix`` (and by the oracle's
``fill_splitmix`` on the host for checks): byte o of a payload arena is
byte (o % 8) of splitmix64 output o // 8 for the config's seed.
Mask keys come from glibc ``random()`` exactly as sequential
``co_ws_frame_serialize`` calls would draw them after ``srandom(key_seed)``.
"""
from __future__ import annotations

import numpy as np

from . import cfws

FRAME_64K = 64 * 1024
CONFIG2 = dict(name="config2", n_frames=65536, frame_size=FRAME_64K,
               payload_seed=0x5EED0002, key_seed=2)


def uniform_batch(n_frames: int, frame_size: int, key_seed: int, opcode: int = cfws.OPCODE_BINARY,
                  mask: bool = True, fin: bool = True) -> np.ndarray:
    """n_frames frames of frame_size bytes, payloads back to back in the arena."""
    d = np.zeros(n_frames, dtype=cfws.DESC_DTYPE)
    d["payload_off"] = np.arange(n_frames, dtype=np.uint64) * np.uint64(frame_size)
    d["payload_size"] = frame_size
    d["fin"] = 1 if fin else 0
    d["opcode"] = opcode
    d["mask"] = 1 if mask else 0
    d["mask_key"] = cfws.draw_mask_keys(n_frames, d["mask"], seed=key_seed)
    return d


def wire_layout(desc: np.ndarray) -> tuple[np.ndarray, int]:
    """Host copy of the serialize plan: (wire offsets, total wire bytes)."""
    sizes = desc["payload_size"].astype(np.uint64) + cfws.header_sizes(desc["payload_size"],
                                                                       desc["mask"])
    offs = np.zeros(len(desc), dtype=np.uint64)
    if len(desc) > 1:
        np.cumsum(sizes[:-1], out=offs[1:])
    return offs, int(sizes.sum())


def round16(n: int) -> int:
    return (n + 15) // 16 * 16
