"""Diagnostic: does the source phase cost the serialize stream anything?
Config 2's frames (65,536 x 64 KiB, masked) serialized from two payload
layouts: "std" (payloads back to back at 64 KiB multiples, so every body's
source runs 14*i mod 16 bytes off its wire position: one aligned load per
lane plus a DPP neighbour block, lane 63 loading the block past its row) and
"aligned" (each payload placed at its wire body offset, phase 0: one load per
lane, no neighbour block). Prints the execute time of each (HIP events, median
of --reps) and checks both wires against each other.

  python tools/phase_probe.py [--reps 20] [--layouts std,aligned]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--frame-size", type=int, default=65536)
    ap.add_argument("--layouts", default="std,aligned")
    a = ap.parse_args()
    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    cfws.init()
    dev = torch.device("cuda", 0)
    F, fs = a.frames, a.frame_size
    base = W.uniform_batch(F, fs, 2)
    offs, wtotal = W.wire_layout(base)
    hs = cfws.header_sizes(base["payload_size"], base["mask"]).astype(np.uint64)
    wire = torch.empty(W.round16(wtotal), dtype=torch.uint8, device=dev)
    stride = int(offs[1] - offs[0]) if F > 1 else fs + int(hs[0])
    assert all(int(offs[i + 1] - offs[i]) == stride for i in (0, F // 2, F - 2)), "uniform frames only"
    # the aligned arena mirrors the wire (payload i at its body offset); std
    # holds the same payload bytes back to back
    aligned = torch.empty(W.round16(wtotal), dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(aligned, 0x5EED0002)
    ref = None
    for layout in a.layouts.split(","):
        d = base.copy()
        if layout == "aligned":
            d["payload_off"] = offs + hs
            payload = aligned
        else:
            payload = torch.empty(F * fs, dtype=torch.uint8, device=dev)
            payload.view(F, fs).copy_(aligned.as_strided((F, fs), (stride, 1), int(hs[0])))
        d_t = cfws.desc_to_device(d, dev)
        ws = cfws.workspace(F, wire.numel(), dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        cfws.serialize_plan(d_t, wire.numel(), tot, ws)
        for _ in range(3):
            cfws.serialize_execute(payload, d_t, wire, ws)
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            cfws.serialize_execute(payload, d_t, wire, ws)
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        torch.cuda.synchronize()
        h = int(torch.sum(wire[:wtotal].view(torch.int64)[: wtotal // 8]).item()) if wtotal % 8 == 0 else None
        same = None
        if ref is None:
            ref = wire[:wtotal].clone()
        else:
            same = bool(torch.equal(ref, wire[:wtotal]))
        med = statistics.median(ms)
        alg = 2 * F * fs + int(hs.sum())
        print(json.dumps({"layout": layout, "execute_ms": round(med, 4),
                          "GBps": round(alg / (med * 1e-3) / 1e9, 1), "same_wire_as_first": same,
                          "sum": h}), flush=True)
        del ws


if __name__ == "__main__":
    main()
