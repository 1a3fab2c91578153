"""TEST INFRASTRUCTURE ONLY -- the codec's parity cases under the library's
launch-time knobs (read once per process from the environment, so
tests/test_knobs.py runs this script once per setting):

  CFWS_EDGE_SPLIT=1     edge chunks as a launch of their own after the stream
  CFWS_EDGE_ORDER=0/1   edge workgroups first / spread through the grid
  CFWS_SMALL=0          small batches on the general plan + execute path
  CFWS_GRID=N           streaming grid capped at N workgroups (grid-stride)
  CFWS_OCC_FRAME_MAX=0  no register-limited residency for small frames
  CFWS_XFORM_LDS=N      the LDS reservation for every mode
  CFWS_PLAN_LDS=N       LDS reserved by the plan kernels
  CFWS_PLAN_SINGLE=0    plans of > 2,048 blocks as reduce / scan / apply
  CFWS_SER_INREG=0      WS serialize edge chunks always by edge workgroups
                        launches instead of the single-pass look-back
  CFWS_FUSED_DESER=0    small-frame deserialize as plan + execute (1, the
                        default: the fused plan + copy)
  CFWS_H2_UNITS_MERGED=0  the HTTP/2 receive's message layout and payload
                        units as two launches (1, the default: one)
  CFWS_SLOTS_WINDOW=0   the fixed-slot receive on its per-frame kernel for
                        every slot size
  CFWS_SLOT_GRID=N      the fixed-slot window kernel as a grid-stride loop
                        over N workgroups

Each case is checked byte for byte against the oracle. Prints "KNOB OK".
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402
import torch  # noqa: E402
from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402


def roundtrip(sizes, rng, seed, align, flags=0, opcodes=None, fins=None, aligned=False):
    n = len(sizes)
    desc = np.zeros(n, dtype=cfws.DESC_DTYPE)
    desc["payload_size"] = sizes
    if aligned:          # 16-aligned payloads (the in-region send edges' condition)
        desc["payload_off"] = np.concatenate([[0], np.cumsum((sizes[:-1] + 15) // 16 * 16)])
    else:
        desc["payload_off"] = np.concatenate([[0], np.cumsum(sizes[:-1])]) + 5
    desc["fin"] = fins if fins is not None else rng.integers(0, 2, n)
    desc["opcode"] = opcodes if opcodes is not None else rng.choice([0, 1, 2, 9, 10], n)
    desc["mask"] = rng.integers(0, 2, n)
    desc["mask_key"] = cfws.draw_mask_keys(n, desc["mask"], seed=seed)
    payload_np = O.fill_splitmix(int(desc["payload_off"][-1]) + int(sizes[-1]) + 32, 0x5EED + seed, 0)
    exp_wire, _ = O.serialize_batch(payload_np, desc.view(O.DESC_DTYPE))
    payload = torch.from_numpy(payload_np).cuda()
    offs, total = W.wire_layout(desc)
    wire = torch.empty(W.round16(total) + 64, dtype=torch.uint8, device="cuda")
    tot = cfws.serialize(payload, cfws.desc_to_device(desc), wire)
    torch.cuda.synchronize()
    assert tot.item() == total == len(exp_wire)
    assert np.array_equal(wire[:total].cpu().numpy(), exp_wire), "serialize != oracle"
    cap = int(sizes.sum()) + align * n + 64
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    d2, st, ptot = cfws.deserialize(wire, total, idx, out, align=align, flags=flags)
    torch.cuda.synchronize()
    e_out, e_d, e_st, e_tot = O.deserialize_batch(exp_wire, offs, align=align, capacity=cap, flags=flags)
    assert ptot.item() == e_tot and np.array_equal(st.cpu().numpy(), e_st)
    assert np.array_equal(out[:e_tot].cpu().numpy(), e_out[:e_tot]), "deserialize != oracle"


def h2_send(sizes, rng, S=16384):
    n = len(sizes)
    payload = O.fill_splitmix(1 << 20, 17, 0)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["payload_size"] = sizes
    d["payload_off"] = rng.integers(0, (1 << 20) - 60000, n).astype(np.uint64)
    d["mask"] = (rng.random(n) < .8).astype(np.uint8)
    d["mask_key"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * d["mask"]
    d["fin"], d["opcode"] = 1, 2
    exp, _ = O.h2_serialize_batch(payload, d, 9, S)
    pay = torch.from_numpy(payload).cuda()
    _, wtotal = W.wire_layout(d)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
    h2 = torch.empty(cfws.h2_wrapped_bound(wire.numel(), n, S), dtype=torch.uint8, device="cuda")
    tot = cfws.h2_serialize(pay, cfws.desc_to_device(d), wire, h2, 9, S)
    torch.cuda.synchronize()
    assert int(tot.item()) == len(exp)
    assert np.array_equal(h2[:len(exp)].cpu().numpy(), exp), "h2 send != oracle"


def main():
    cfws.init()
    rng = np.random.default_rng(11)
    # mixed sizes: fast / two-frame / general regions, edges, 64-bit lengths
    sizes = rng.choice([0, 1, 3, 125, 126, 1000, 4096, 65535, 65536, 70000], size=3000)
    for align in (1, 16):
        roundtrip(sizes, rng, 1, align)
    # 1 KiB frames in a large batch (spread edges, register-limited residency)
    roundtrip(np.full(20000, 1024), rng, 2, 16, opcodes=np.full(20000, 1), fins=np.ones(20000))
    # 600 K tiny frames: plans of > 2,048 blocks (single-pass unless CFWS_PLAN_SINGLE=0)
    roundtrip(rng.integers(0, 31, 600000), rng, 4, 1)
    # 80..2,000-byte payloads at 16-aligned offsets (bound 3,584): in-region send edge chunks
    # unless CFWS_SER_INREG=0 or CFWS_EDGE_SPLIT=1 (reduce + apply plan, then
    # the single-pass plan)
    roundtrip(rng.integers(80, 2001, 20000), rng, 5, 16, aligned=True)
    roundtrip(rng.integers(80, 200, 600000), rng, 6, 1, aligned=True)
    # WebSocket over HTTP/2, DATA frames all over 4 KiB + 32: the fused
    # send's in-region edge chunks unless CFWS_H2_INREG=0 or CFWS_EDGE_SPLIT=1
    h2_send(rng.integers(4200, 60000, 1500), rng)
    # small frames at 16-byte slots: the fused deserialize (<= 512 wire bytes
    # per frame; CFWS_FUSED_DESER=0: plan + execute)
    roundtrip(rng.integers(0, 600, 200000), rng, 7, 16)
    if "CFWS_FUSED_DESER" in os.environ:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import test_gpu_batch as T
        for align in (16, 64):
            T.test_fused_deserialize_mixed_and_errors(align)
        # frame starts out of order and reversed
        import random
        w, _ = T.wire_stream(random.Random(8), 30000, sizes=list(range(0, 1000, 7)))
        offs, consumed = O.index_frames(w, 40000)
        assert consumed == len(w)
        perm = np.random.default_rng(9).permutation(len(offs))
        T.check_deserialize(w, offs[perm], align=16)
        T.check_deserialize(w, offs[::-1].copy(), align=16)
    if "CFWS_H2_UNITS_MERGED" in os.environ:
        # the HTTP/2 receive with its message layout and units as two launches
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import test_h2 as T2
        T2.test_gpu_h2_roundtrip_random(16384)
        T2.test_gpu_h2_deserialize_headers_across_data_frames(13)
        T2.test_gpu_h2_rows_past_message_count_are_empty(2)
        T2.test_gpu_h2_long_messages(1000)
    if "CFWS_SLOTS_WINDOW" in os.environ or "CFWS_SLOT_GRID" in os.environ:
        # the fixed-slot receive: every slot size on the per-frame kernel
        # (CFWS_SLOTS_WINDOW=0), or the window kernel as a grid-stride loop
        # over a capped grid (CFWS_SLOT_GRID), over guarded arenas
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import test_gpu_slots as TS
        if TS._glib().guard_supported():
            bufs = []

            def make(n, flush_end=True):
                b = TS.GuardBuf(n, flush_end, TS.SENT)
                bufs.append(b)
                return b
            for slot in (16, 256, 992, 1504, 4064, 8160):
                for seed in (21, 22):
                    TS.test_slots_mixed(make, seed, slot)
            TS.test_slots_capacity_cuts(make)
            TS.test_slots_truncated_wire(make)
            TS.test_slots_any_index(make)
            for fs in (256, 1000, 3072):
                TS.test_slots_uniform(make, fs)
            torch.cuda.synchronize()
            for b in bufs:
                b.free()
    # a small batch (single-launch path unless CFWS_SMALL=0)
    roundtrip(np.full(256, 1000), rng, 3, 16)
    # fragments + pings, reassembled (two passes, pass-1 capped grid)
    desc, msgs = W.zipf_batch(48 << 20, 0x5EED0003, 3, ping_every=5)
    arena = O.splitmix_words(0x5EED0003, 0, (msgs["arena_bytes"] + 7) // 8).view(np.uint8)[:msgs["arena_bytes"]]
    exp_wire, d2 = O.serialize_batch(arena, desc.view(O.DESC_DTYPE))
    wire = torch.from_numpy(exp_wire).cuda()
    cap = len(arena) + 64
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    idx = torch.from_numpy(d2["wire_off"].astype(np.int64)).cuda()
    _, st, ptot = cfws.deserialize(wire, len(exp_wire), idx, out, flags=cfws.DESERIALIZE_REASSEMBLE)
    torch.cuda.synchronize()
    e_out, _, e_st, e_tot = O.deserialize_batch(exp_wire, d2["wire_off"], capacity=cap,
                                                flags=O.DESERIALIZE_REASSEMBLE)
    assert ptot.item() == e_tot and np.array_equal(st.cpu().numpy(), e_st)
    assert np.array_equal(out[:e_tot].cpu().numpy(), e_out[:e_tot]), "reassembly != oracle"
    print("KNOB OK", {k: v for k, v in os.environ.items() if k.startswith("CFWS_")}, flush=True)


if __name__ == "__main__":
    main()
