#!/usr/bin/env python3
"""bench_e2e.py -- the PCIe-inclusive rate of the codec.

coldforce's frames start and end in host memory (socket buffers), so besides
the device-resident metric (bench.py) this measures the host-to-host rate of
the same work through cfws_pipeline_* (pinned host buffers, chunks of
frames, H2D / plan + kernels / D2H overlapped across `depth` streams):

  serialize:   host payload arena -> host wire arena   (client mask)
  deserialize: host wire arena    -> host payload arena (server unmask)

It also times plain pinned H2D and D2H copies of the same size (the PCIe
ceiling). Prints one JSON line. Never part of the device-resident `value`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["config2", "config3"], default="config2")
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--frame-size", type=int, default=65536)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W

    cfws.init()
    if args.workload == "config3":
        c3 = W.CONFIG3
        desc, msgs = W.zipf_batch(c3["target_bytes"], c3["seed"], c3["key_seed"])
        nbytes, seed = int(msgs["arena_bytes"]), c3["seed"]
    else:
        desc = W.uniform_batch(args.frames, args.frame_size, 2)
        nbytes, seed = args.frames * args.frame_size, 0x5EED0002
    offs, wire_total = W.wire_layout(desc)

    payload = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    wire = torch.empty(wire_total + 64, dtype=torch.uint8, pin_memory=True)
    back = torch.empty(nbytes + 16 * len(desc) + 64, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(dev, seed)
    torch.cuda.synchronize()

    # PCIe ceiling: plain pinned copies of the payload size
    t0 = time.perf_counter()
    for _ in range(args.reps):
        payload.copy_(dev, non_blocking=True)
    torch.cuda.synchronize()
    d2h = args.reps * nbytes / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    for _ in range(args.reps):
        dev.copy_(payload, non_blocking=True)
    torch.cuda.synchronize()
    h2d = args.reps * nbytes / (time.perf_counter() - t0) / 1e9

    pl = cfws.Pipeline(chunk_bytes=args.chunk_mib << 20, max_frames=1 << 16, depth=args.depth)
    d = desc.copy()
    pl.serialize(payload.data_ptr(), d, wire.data_ptr(), wire.numel())          # warm-up
    t0 = time.perf_counter()
    for _ in range(args.reps):
        d = desc.copy()
        tot = pl.serialize(payload.data_ptr(), d, wire.data_ptr(), wire.numel())
    t_ser = (time.perf_counter() - t0) / args.reps
    pl.deserialize(wire.data_ptr(), tot, offs, back.data_ptr(), back.numel(), align=1)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        dd, st, ptot = pl.deserialize(wire.data_ptr(), tot, offs, back.data_ptr(), back.numel(),
                                      align=1)
    t_de = (time.perf_counter() - t0) / args.reps
    pl.close()
    ok = (tot == wire_total and ptot == nbytes and bool((st == 0).all())
          and torch.equal(back[:nbytes], payload))
    line = {
        "what": "host-to-host (PCIe-inclusive) codec rate through cfws_pipeline_*",
        "workload": args.workload, "frames": len(desc), "payload_bytes": nbytes,
        "wire_bytes": wire_total, "chunk_mib": args.chunk_mib, "depth": args.depth,
        "serialize_s": round(t_ser, 4), "deserialize_s": round(t_de, 4),
        "serialize_GiBps": round(nbytes / t_ser / GIB, 2),
        "deserialize_GiBps": round(nbytes / t_de / GIB, 2),
        "round_trip_GiBps": round(2 * nbytes / (t_ser + t_de) / GIB, 2),
        "pinned_h2d_GBps": round(h2d, 1), "pinned_d2h_GBps": round(d2h, 1),
        "verified": ok,
    }
    print(json.dumps(line), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
