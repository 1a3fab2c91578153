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


def host_buffer(args, n):
    import torch

    from coldforce_amd import cfws
    if args.host == "mapped":
        return cfws.mapped_host(n)[:n]
    return torch.empty(n, dtype=torch.uint8, pin_memory=True)


def e2e_h2(args):
    """Config 5 host to host: payload (pinned) -> H2D -> WS serialize + HTTP/2
    DATA wrap -> D2H DATA stream, and back (H2D -> unwrap + pool + unmask ->
    D2H), chunks of frames overlapped on `depth` streams."""
    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    F = args.frames
    fs = 16376 if args.frame_size == 65536 and "--frame-size" not in sys.argv else args.frame_size
    S = cfws.H2_DEFAULT_MAX_FRAME_SIZE
    CF = max(1, (args.chunk_mib << 20) // fs)           # frames per chunk
    desc = W.uniform_batch(F, fs, 5)
    hs = int(cfws.header_sizes(np.array([fs]), np.array([1]))[0])
    Wf = fs + hs
    k = -(-Wf // S)
    Hf = Wf + 9 * k                                       # DATA-stream bytes per WS frame
    payload = host_buffer(args, F * fs)
    h2 = host_buffer(args, F * Hf)
    back = host_buffer(args, F * fs)
    # D2H by kernel (cfws_copy_to_host) only into mapped memory and only when
    # --d2h kernel: this harness enqueues every chunk without host
    # back-pressure, and there SDMA measured faster both ways (serialize 38
    # vs 33 GiB/s), so its auto is SDMA (the C pipeline's auto differs)
    ser_kernel = de_kernel = args.host == "mapped" and args.d2h == "kernel"
    dev = torch.empty(F * fs, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(dev, 0x5EED0005)
    payload.copy_(dev)
    del dev
    streams = [torch.cuda.Stream() for _ in range(args.depth)]
    chunks = [(c0, min(F, c0 + CF)) for c0 in range(0, F, CF)]
    descs = []
    for c0, c1 in chunks:
        d = desc[c0:c1].copy()
        d["payload_off"] -= np.uint64(c0 * fs)
        descs.append(cfws.desc_to_device(d))
    per = np.arange(CF, dtype=np.uint64) * np.uint64(Hf)
    starts = (per[:, None] + (np.arange(k, dtype=np.uint64) * np.uint64(S + 9))[None, :]).reshape(-1)
    slot = []
    for s in range(args.depth):
        with torch.cuda.stream(streams[s]):
            pay_d = torch.empty(CF * fs + 16, dtype=torch.uint8, device="cuda")
            wire_d = torch.empty(CF * Wf + 32, dtype=torch.uint8, device="cuda")
            h2_d = torch.empty(cfws.h2_wrapped_bound(wire_d.numel(), CF, S), dtype=torch.uint8, device="cuda")
            pool_d = torch.empty(CF * Wf + 16, dtype=torch.uint8, device="cuda")
            back_d = torch.empty(CF * fs + 64, dtype=torch.uint8, device="cuda")
            ws_s = torch.empty(cfws.lib().cfws_h2_serialize_workspace_size(CF, wire_d.numel(), h2_d.numel(), S),
                               dtype=torch.uint8, device="cuda")
            ws_d = torch.empty(cfws.lib().cfws_h2_deserialize_workspace_size(CF * k, pool_d.numel(),
                                                                            back_d.numel()),
                               dtype=torch.uint8, device="cuda")
            idx = torch.from_numpy(starts.astype(np.int64)).cuda()
            tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        slot.append((pay_d, wire_d, h2_d, pool_d, back_d, ws_s, ws_d, idx, tot))
    torch.cuda.synchronize()

    # H2D copies go in chunk order on one copy stream, each waiting only for
    # its slot's previous kernels (the input staging free), as in
    # cfws_pipeline_*: behind the slot's D2H on its own stream they would
    # alternate with the D2H bursts instead of overlapping them.
    st_in = torch.cuda.Stream()
    ev_in = [torch.cuda.Event() for _ in range(args.depth)]
    ev_exec = [torch.cuda.Event() for _ in range(args.depth)]
    for s in range(args.depth):
        ev_exec[s].record(streams[s])

    def to_device(dst, src, s):
        st_in.wait_event(ev_exec[s])
        with torch.cuda.stream(st_in):
            dst.copy_(src, non_blocking=True)
        ev_in[s].record(st_in)

    def ser():
        for c, (c0, c1) in enumerate(chunks):
            s = c % args.depth
            st = streams[s]
            pay_d, wire_d, h2_d, _, _, ws_s, _, _, tot = slot[s]
            to_device(pay_d[:(c1 - c0) * fs], payload[c0 * fs:c1 * fs], s)
            st.wait_event(ev_in[s])
            with torch.cuda.stream(st):
                cfws.h2_serialize(pay_d, descs[c], wire_d, h2_d, 1, S, ws_s, tot, stream=st)
                ev_exec[s].record(st)
                if ser_kernel:
                    cfws.copy_to_host(h2_d, h2[c0 * Hf:].data_ptr(), (c1 - c0) * Hf, stream=st)
                else:
                    h2[c0 * Hf:c1 * Hf].copy_(h2_d[:(c1 - c0) * Hf], non_blocking=True)
        torch.cuda.synchronize()

    def de():
        ok = True

        def fetch(c):
            c0, c1 = chunks[c]
            to_device(slot[c % args.depth][2][:(c1 - c0) * Hf], h2[c0 * Hf:c1 * Hf], c % args.depth)

        # h2_deserialize synchronises its stream (message count): the next
        # depth - 1 chunks' H2D are queued before each call
        for c in range(min(args.depth - 1, len(chunks))):
            fetch(c)
        for c, (c0, c1) in enumerate(chunks):
            if c + args.depth - 1 < len(chunks):
                fetch(c + args.depth - 1)
            s = c % args.depth
            st = streams[s]
            _, _, h2_d, pool_d, back_d, _, ws_d, idx, _ = slot[s]
            n = c1 - c0
            st.wait_event(ev_in[s])
            with torch.cuda.stream(st):
                hs_, md, ms, ptot, m = cfws.h2_deserialize(h2_d, n * Hf, idx[:n * k], pool_d, back_d,
                                                           S, align=1, ws_t=ws_d, stream=st)
                ev_exec[s].record(st)
                if de_kernel:
                    cfws.copy_to_host(back_d, back[c0 * fs:].data_ptr(), n * fs, stream=st)
                else:
                    back[c0 * fs:c1 * fs].copy_(back_d[:n * fs], non_blocking=True)
                ok = ok and m == n
        torch.cuda.synchronize()
        return ok

    ser()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ser()
    t_ser = (time.perf_counter() - t0) / args.reps
    de()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ok = de()
    t_de = (time.perf_counter() - t0) / args.reps
    nbytes = F * fs
    ok = ok and torch.equal(back, payload)
    line = {"what": "config 5 host-to-host (PCIe-inclusive): WS over HTTP/2 DATA frames",
            "workload": "config5", "frames": F, "payload_bytes": nbytes, "h2_bytes": F * Hf,
            "data_frames": F * k, "chunk_frames": CF, "depth": args.depth,
            "serialize_s": round(t_ser, 4), "deserialize_s": round(t_de, 4),
            "serialize_GiBps": round(nbytes / t_ser / GIB, 2),
            "deserialize_GiBps": round(nbytes / t_de / GIB, 2),
            "round_trip_GiBps": round(2 * nbytes / (t_ser + t_de) / GIB, 2), "host": args.host, "d2h": args.d2h,
            "verified": ok}
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
    args = ap.parse_args()

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
        "host": args.host, "d2h": args.d2h,
        "pinned_h2d_GBps": round(h2d, 1), "pinned_d2h_GBps": round(d2h, 1),
        "verified": ok,
    }
    print(json.dumps(line), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
