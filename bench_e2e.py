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


def bind_numa_node(node: int) -> list[int]:
    """Restricts this process (every thread it starts from here on) to the
    CPUs of NUMA node `node`, read from sysfs. Called before torch / HIP load,
    so the pipeline's threads and the first touch of the host arenas stay on
    that node (no numactl on the image)."""
    cpus = []
    with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
        for part in f.read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.extend(range(int(lo), int(hi or lo) + 1))
    os.sched_setaffinity(0, cpus)
    return cpus


def host_buffer(args, n):
    import torch

    from coldforce_amd import cfws
    if args.host == "mapped":
        return cfws.mapped_host(n)[:n]
    return torch.empty(n, dtype=torch.uint8, pin_memory=True)


def timed(fn, reps: int) -> float:
    """Median wall time of reps calls (each synchronous on return)."""
    import numpy as np
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def e2e_h2(args):
    """Config 5 host to host through cfws_pipeline_h2_*: payload arena ->
    WS serialize + HTTP/2 DATA wrap -> DATA-frame stream (send), and DATA
    stream -> pooled messages -> WS deserialize -> payload arena (receive),
    chunked over `depth` slots with H2D / kernels / D2H overlapped."""
    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    F = args.frames
    fs = 16376 if args.frame_size == 65536 and "--frame-size" not in sys.argv else args.frame_size
    S = cfws.H2_DEFAULT_MAX_FRAME_SIZE
    desc = W.uniform_batch(F, fs, 5)
    hs = int(cfws.header_sizes(np.array([fs]), np.array([1]))[0])
    Wf = fs + hs
    k = -(-Wf // S)
    Hf = Wf + 9 * k                                       # DATA-stream bytes per WS frame
    payload = host_buffer(args, F * fs)
    h2 = host_buffer(args, F * Hf)
    back = host_buffer(args, F * fs + 64)
    dev = torch.empty(F * fs, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(dev, 0x5EED0005)
    payload.copy_(dev)
    del dev
    per = np.arange(F, dtype=np.uint64) * np.uint64(Hf)
    index = (per[:, None] + (np.arange(k, dtype=np.uint64) * np.uint64(S + 9))[None, :]).reshape(-1)
    pl = cfws.Pipeline(chunk_bytes=args.chunk_mib << 20, max_frames=1 << 16, depth=args.depth,
                       d2h=args.d2h)

    def ser():
        return pl.h2_serialize(payload.data_ptr(), desc, h2.data_ptr(), h2.numel(), 1, S)

    def de():
        return pl.h2_deserialize(h2.data_ptr(), F * Hf, index, back.data_ptr(), back.numel(), S,
                                 align=1)

    assert ser() == F * Hf
    t_ser = timed(ser, args.reps)
    st, md, ms, tot = de()
    t_de = timed(de, args.reps)
    nbytes = F * fs
    ok = (len(md) == F and tot == nbytes and bool((st == 0).all()) and bool((ms == 0).all())
          and torch.equal(back[:nbytes], payload[:nbytes]))
    pl.close()
    line = {"what": "config 5 host-to-host (PCIe-inclusive): WS over HTTP/2 DATA frames, cfws_pipeline_h2_*",
            "workload": "config5", "frames": F, "payload_bytes": nbytes, "h2_bytes": F * Hf,
            "data_frames": F * k, "chunk_mib": args.chunk_mib, "depth": args.depth,
            "serialize_s": round(t_ser, 4), "deserialize_s": round(t_de, 4),
            "serialize_GiBps": round(nbytes / t_ser / GIB, 2),
            "deserialize_GiBps": round(nbytes / t_de / GIB, 2),
            "round_trip_GiBps": round(2 * nbytes / (t_ser + t_de) / GIB, 2), "host": args.host,
            "d2h": args.d2h, "numa_node": args.numa_node,
            "timing": f"median of {args.reps} reps after one warm-up", "verified": ok}
    print(json.dumps(line), flush=True)
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["config2", "config3", "config5"], default="config2")
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--frame-size", type=int, default=65536)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--d2h", choices=["auto", "dma", "kernel"], default="auto",
                    help="the pipeline's D2H mode into mapped arenas (cfws_pipeline_set_d2h): "
                         "auto = kernel for serialize, SDMA for deserialize")
    ap.add_argument("--host", choices=["mapped", "torch"], default="mapped",
                    help="host arenas: mapped pinned memory (hipHostMallocMapped; the D2H leg "
                         "may be a kernel writing it, cfws_copy_to_host) or torch pinned memory "
                         "(the D2H leg is an SDMA copy)")
    ap.add_argument("--numa-node", type=int, default=-1,
                    help="bind to this NUMA node's CPUs before HIP loads (-1: the OS's choice)")
    args = ap.parse_args()
    if args.numa_node >= 0:
        bind_numa_node(args.numa_node)

    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W

    cfws.init()
    if args.workload == "config5":
        sys.exit(e2e_h2(args))
    if args.workload == "config3":
        c3 = W.CONFIG3
        desc, msgs = W.zipf_batch(c3["target_bytes"], c3["seed"], c3["key_seed"])
        nbytes, seed = int(msgs["arena_bytes"]), c3["seed"]
    else:
        desc = W.uniform_batch(args.frames, args.frame_size, 2)
        nbytes, seed = args.frames * args.frame_size, 0x5EED0002
    offs, wire_total = W.wire_layout(desc)

    payload = host_buffer(args, nbytes)
    wire = host_buffer(args, wire_total + 64)
    back = host_buffer(args, nbytes + 16 * len(desc) + 64)
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

    pl = cfws.Pipeline(chunk_bytes=args.chunk_mib << 20, max_frames=1 << 16, depth=args.depth,
                       d2h=args.d2h)
    d = desc.copy()
    pl.serialize(payload.data_ptr(), d, wire.data_ptr(), wire.numel())          # warm-up
    ts = []
    for _ in range(args.reps):
        d = desc.copy()
        t0 = time.perf_counter()
        tot = pl.serialize(payload.data_ptr(), d, wire.data_ptr(), wire.numel())
        ts.append(time.perf_counter() - t0)
    t_ser = float(np.median(ts))
    pl.deserialize(wire.data_ptr(), tot, offs, back.data_ptr(), back.numel(), align=1)
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        dd, st, ptot = pl.deserialize(wire.data_ptr(), tot, offs, back.data_ptr(), back.numel(),
                                      align=1)
        ts.append(time.perf_counter() - t0)
    t_de = float(np.median(ts))
    ok = (tot == wire_total and ptot == nbytes and bool((st == 0).all())
          and torch.equal(back[:nbytes], payload))
    # the receive loop: host frame walk (cfws_index_frames) + the same pipeline
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        dr, sr, consumed, stop, rtot = pl.receive(wire.data_ptr(), 0, tot, back.data_ptr(),
                                                  back.numel(), max_frames=len(desc), align=1)
        ts.append(time.perf_counter() - t0)
    t_rx = float(np.median(ts))
    ok = ok and consumed == tot and stop == 0 and rtot == nbytes and len(dr) == len(desc)
    pl.close()
    line = {
        "what": "host-to-host (PCIe-inclusive) codec rate through cfws_pipeline_*",
        "workload": args.workload, "frames": len(desc), "payload_bytes": nbytes,
        "wire_bytes": wire_total, "chunk_mib": args.chunk_mib, "depth": args.depth,
        "serialize_s": round(t_ser, 4), "deserialize_s": round(t_de, 4),
        "serialize_GiBps": round(nbytes / t_ser / GIB, 2),
        "deserialize_GiBps": round(nbytes / t_de / GIB, 2),
        "round_trip_GiBps": round(2 * nbytes / (t_ser + t_de) / GIB, 2),
        "receive_s": round(t_rx, 4), "receive_GiBps": round(nbytes / t_rx / GIB, 2),
        "timing": f"median of {args.reps} reps after one warm-up",
        "host": args.host, "d2h": args.d2h, "numa_node": args.numa_node,
        "pinned_h2d_GBps": round(h2d, 1), "pinned_d2h_GBps": round(d2h, 1),
        "verified": ok,
    }
    print(json.dumps(line), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
