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


# ---- config 3: Zipf messages split into continuation fragments --------------

CONFIG3 = dict(name="config3", target_bytes=4 << 30, seed=0x5EED0003, key_seed=3)
ZIPF_KMAX = 16384           # message length = 64 * k, k in [1, 16384] (64 B .. 1 MiB)
ZIPF_S = 1.1


def _uniform(seed: int, idx: np.ndarray) -> np.ndarray:
    """Deterministic uniforms in [0, 1): splitmix64(seed, idx) >> 11 * 2^-53."""
    i = idx.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def zipf_message_sizes(n: int, seed: int) -> np.ndarray:
    """n message lengths 64*k with P(k) ~ k^-1.1, k in [1, 16384]."""
    k = np.arange(1, ZIPF_KMAX + 1, dtype=np.float64)
    cdf = np.cumsum(k ** -ZIPF_S)
    cdf /= cdf[-1]
    u = _uniform(seed, np.arange(n, dtype=np.uint64) * np.uint64(16))
    kk = np.searchsorted(cdf, u, side="right") + 1
    return (64 * np.minimum(kk, ZIPF_KMAX)).astype(np.uint64)


def zipf_batch(target_bytes: int, seed: int = CONFIG3["seed"], key_seed: int = CONFIG3["key_seed"],
               ping_every: int = 0, max_messages: int | None = None):
    """Messages until the payload reaches target_bytes; each split into 1-8
    fragments at random cut points (first TEXT or BINARY fin=0, middle
    CONTINUATION fin=0, last CONTINUATION fin=1, or one fin=1 frame when
    unfragmented); all frames client-masked. With ping_every = p > 0 a masked
    PING (8-byte payload) is interleaved after every p-th non-final fragment
    (control frames may interleave a fragmented message, RFC 6455 5.4).
    Returns (desc, messages) where messages is a dict of numpy arrays:
    off, len, opcode, first_frame, n_frames. The payload arena holds the
    messages back to back, then the ping payloads; its size is
    messages['arena_bytes']."""
    # sizes: draw in blocks until the target is met
    n_guess = max(16, int(target_bytes / 60000))
    sizes = zipf_message_sizes(n_guess, seed)
    while sizes.sum() < target_bytes and (max_messages is None or len(sizes) < max_messages):
        n_guess *= 2
        sizes = zipf_message_sizes(n_guess, seed)
    csum = np.cumsum(sizes)
    n_msg = int(np.searchsorted(csum, target_bytes) + 1)
    n_msg = min(n_msg, len(sizes))
    if max_messages is not None:
        n_msg = min(n_msg, max_messages)
    sizes = sizes[:n_msg]
    mid = np.arange(n_msg, dtype=np.uint64) * np.uint64(16)
    nfrag = 1 + np.floor(_uniform(seed, mid + np.uint64(1)) * 8).astype(np.int64)
    opcode0 = np.where(_uniform(seed, mid + np.uint64(2)) < 0.5, 1, 2).astype(np.uint8)
    moff = np.zeros(n_msg, dtype=np.uint64)
    if n_msg > 1:
        np.cumsum(sizes[:-1], out=moff[1:])
    data_bytes = int(sizes.sum())

    if not ping_every:
        return _zipf_frames(sizes, nfrag, opcode0, moff, seed, key_seed)

    rows = []   # (payload_off, size, fin, opcode)
    first_frame = np.zeros(n_msg, dtype=np.int64)
    n_frames = np.zeros(n_msg, dtype=np.int64)
    ping_bytes = 0
    ping_count = 0
    frag_counter = 0
    for m in range(n_msg):
        L, f = int(sizes[m]), int(nfrag[m])
        if f > 1:
            u = _uniform(seed, np.uint64(m * 16 + 3) + np.arange(f - 1, dtype=np.uint64))
            cuts = np.sort(1 + np.floor(u * (L - 1)).astype(np.int64))
            bounds = np.concatenate([[0], cuts, [L]])
        else:
            bounds = np.array([0, L])
        first_frame[m] = len(rows)
        for j in range(f):
            a, b = int(bounds[j]), int(bounds[j + 1])
            op = int(opcode0[m]) if j == 0 else 0
            rows.append((int(moff[m]) + a, b - a, 1 if j == f - 1 else 0, op))
            frag_counter += 1
            if ping_every and j < f - 1 and frag_counter % ping_every == 0:
                rows.append((data_bytes + ping_bytes, 8, 1, 0x9))
                ping_bytes += 8
                ping_count += 1
        n_frames[m] = len(rows) - first_frame[m]
    d = np.zeros(len(rows), dtype=cfws.DESC_DTYPE)
    arr = np.array(rows, dtype=np.uint64)
    d["payload_off"] = arr[:, 0]
    d["payload_size"] = arr[:, 1]
    d["fin"] = arr[:, 2].astype(np.uint8)
    d["opcode"] = arr[:, 3].astype(np.uint8)
    d["mask"] = 1
    d["mask_key"] = cfws.draw_mask_keys(len(rows), seed=key_seed)
    messages = dict(off=moff, len=sizes, opcode=opcode0, first_frame=first_frame,
                    n_frames=n_frames, arena_bytes=data_bytes + ping_bytes,
                    data_bytes=data_bytes, pings=ping_count)
    return d, messages


def _zipf_frames(sizes, nfrag, opcode0, moff, seed: int, key_seed: int):
    """zipf_batch's fragmenting without PINGs, vectorised over messages (the
    same cut points and frame rows as its per-message loop, which an 8-GPU
    global batch of 2.4 M frames makes too slow)."""
    n_msg = len(sizes)
    f = nfrag.astype(np.int64)
    L = sizes.astype(np.int64)
    n_frames = f.copy()
    first_frame = np.zeros(n_msg, dtype=np.int64)
    if n_msg > 1:
        np.cumsum(f[:-1], out=first_frame[1:])
    n_rows = int(f.sum())
    # cut j of message m (j < f-1): 1 + floor(u(m*16 + 3 + j) * (L-1)), sorted per message
    ncut = f - 1
    cut_msg = np.repeat(np.arange(n_msg, dtype=np.int64), ncut)
    cut_j = np.arange(int(ncut.sum()), dtype=np.int64) - np.repeat(np.cumsum(ncut) - ncut, ncut)
    u = _uniform(seed, cut_msg.astype(np.uint64) * np.uint64(16) + np.uint64(3) + cut_j.astype(np.uint64))
    cuts = 1 + np.floor(u * (L[cut_msg] - 1).astype(np.float64)).astype(np.int64)
    cuts = cuts[np.lexsort((cuts, cut_msg))]
    # row r of message m = fragment j: [bound j, bound j+1) with bounds 0, cuts.., L
    row_msg = np.repeat(np.arange(n_msg, dtype=np.int64), f)
    row_j = np.arange(n_rows, dtype=np.int64) - first_frame[row_msg]
    cut_base = (np.cumsum(ncut) - ncut)[row_msg]           # first cut of the row's message
    cuts = np.append(cuts, 0)                              # sentinel for rows without a cut
    first, last = row_j == 0, row_j == f[row_msg] - 1
    lo = np.where(first, 0, cuts[np.where(first, len(cuts) - 1, cut_base + row_j - 1)])
    hi = np.where(last, L[row_msg], cuts[np.where(last, len(cuts) - 1, cut_base + row_j)])
    d = np.zeros(n_rows, dtype=cfws.DESC_DTYPE)
    d["payload_off"] = moff[row_msg] + lo.astype(np.uint64)
    d["payload_size"] = (hi - lo).astype(np.uint64)
    d["fin"] = last.astype(np.uint8)
    d["opcode"] = np.where(row_j == 0, opcode0[row_msg], 0).astype(np.uint8)
    d["mask"] = 1
    d["mask_key"] = cfws.draw_mask_keys(n_rows, seed=key_seed)
    data_bytes = int(sizes.sum())
    messages = dict(off=moff, len=sizes, opcode=opcode0, first_frame=first_frame,
                    n_frames=n_frames, arena_bytes=data_bytes, data_bytes=data_bytes, pings=0)
    return d, messages
