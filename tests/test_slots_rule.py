"""The fixed-slot layout as include/cfws.h states it for
cfws_deserialize_slots, checked on the CPU against hand-built frames: the
expectation the GPU tests compare with (test_gpu_slots.expect_slots) must
itself say what the header says. Slot i starts at i * slot; a COMPLETE
frame's payload is unmasked there, then zeros up to its 16-byte round-up
(cut at the capacity); a payload longer than the slot, or ending past the
capacity, is OUT_OF_MEMORY and its slot is not written; every other byte
keeps what was there."""
import numpy as np

import oracle as O
from test_gpu_slots import SENT, expect_slots


def _wire(frames):
    """frames: (payload bytes, mask key or None) -> (wire, starts)."""
    n = len(frames)
    sizes = np.array([len(p) for p, _ in frames], dtype=np.uint64)
    arena = np.frombuffer(b"".join(p for p, _ in frames), np.uint8).copy()
    desc = np.zeros(n, dtype=O.DESC_DTYPE)
    desc["payload_size"] = sizes
    desc["payload_off"] = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64) if n else []
    desc["fin"] = 1
    desc["opcode"] = 2
    desc["mask"] = [k is not None for _, k in frames]
    desc["mask_key"] = [k or 0 for _, k in frames]
    wire, _ = O.serialize_batch(arena if arena.size else np.zeros(1, np.uint8), desc)
    starts, _ = O.index_frames(wire, n + 1)
    return wire, starts


def _unmask(p, key):
    k = np.frombuffer(int(key).to_bytes(4, "little"), np.uint8)
    a = np.frombuffer(p, np.uint8)
    return a ^ np.resize(k, a.size)


def test_layout_padding_and_untouched_bytes():
    frames = [(bytes(range(20)), 0x11223344), (b"", None), (bytes(range(100, 133)), None)]
    wire, starts = _wire(frames)
    slot = 48
    arena, d, st, tot = expect_slots(wire, len(wire), starts, slot, 3 * slot)
    assert list(st) == [O.PARSE_COMPLETE] * 3 and tot == 3 * slot
    assert list(d["payload_off"]) == [0, 48, 96]
    # frame 0: 20 payload bytes (masked on the wire, unmasked here), zeros to 32
    assert np.array_equal(arena[0:20], np.frombuffer(bytes(range(20)), np.uint8))
    assert (arena[20:32] == 0).all() and (arena[32:48] == SENT).all()
    # frame 1: empty, its slot untouched
    assert (arena[48:96] == SENT).all()
    # frame 2: 33 bytes, zeros to 48 (= its 16-byte round-up)
    assert np.array_equal(arena[96:129], np.frombuffer(bytes(range(100, 133)), np.uint8))
    assert (arena[129:144] == 0).all()
    assert _unmask(bytes(range(20)), 0x11223344).size == 20


def test_out_of_memory_by_slot_and_by_capacity():
    frames = [(bytes(40), None), (bytes(10), None), (bytes(16), None)]
    wire, starts = _wire(frames)
    # slot 32: frame 0 (40 B) does not fit its slot
    arena, d, st, tot = expect_slots(wire, len(wire), starts, 32, 96)
    assert list(st) == [O.ERROR_OUT_OF_MEMORY, O.PARSE_COMPLETE, O.PARSE_COMPLETE]
    assert (arena[0:32] == SENT).all() and tot == 96
    # capacity 70: frame 2 starts at 64, its 16 bytes end past 70
    arena, d, st, tot = expect_slots(wire, len(wire), starts, 32, 70)
    assert list(st) == [O.ERROR_OUT_OF_MEMORY, O.PARSE_COMPLETE, O.ERROR_OUT_OF_MEMORY]
    assert tot == 70 and (arena[64:80] == SENT).all()
    # capacity 40: frame 1's payload would end at byte 42, past the
    # capacity, so the whole frame is OUT_OF_MEMORY (nothing is cut)
    arena, d, st, tot = expect_slots(wire, len(wire), starts, 32, 40)
    assert st[1] == O.ERROR_OUT_OF_MEMORY and tot == 40


def test_padding_cut_at_the_capacity():
    frames = [(bytes(range(1, 11)), None)]
    wire, starts = _wire(frames)
    arena, d, st, tot = expect_slots(wire, len(wire), starts, 16, 12)
    assert st[0] == O.PARSE_COMPLETE and tot == 12
    assert np.array_equal(arena[:10], np.arange(1, 11, dtype=np.uint8))
    assert (arena[10:12] == 0).all() and (arena[12:16] == SENT).all()


def test_non_complete_frames_keep_their_slots():
    frames = [(bytes(30), None), (bytes(30), None)]
    wire, starts = _wire(frames)
    cut = int(starts[1]) + 5                      # frame 1 is MORE_DATA
    arena, d, st, tot = expect_slots(wire, cut, starts, 32, 64)
    assert list(st) == [O.PARSE_COMPLETE, O.PARSE_MORE_DATA]
    assert (arena[32:64] == SENT).all() and list(d["payload_off"]) == [0, 32]
