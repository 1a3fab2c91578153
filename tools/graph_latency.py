"""Small-batch cost of the batch codec, eager vs replayed HIP graphs
(cfws_graph_*): a round trip = serialize (client mask) + deserialize
(server unmask) of n frames of `size` bytes, device resident.
  latency_us:   one round trip, synchronised every iteration (median)
  pipelined_us: round trips enqueued back to back, one sync at the end
Prints one JSON line per (n, mode)."""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,16,256,4096")
    ap.add_argument("--frame-size", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--stream", choices=["default", "created"], default="created",
                    help="torch's default (null) stream or a created one")
    a = ap.parse_args()
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    cfws.init()
    fs = a.frame_size
    if a.stream == "created":
        torch.cuda.set_stream(torch.cuda.Stream())
    for n in [int(x) for x in a.sizes.split(",")]:
        desc = W.uniform_batch(n, fs, 1, opcode=cfws.OPCODE_TEXT)
        offs, wtotal = W.wire_layout(desc)
        pay = torch.empty(W.round16(n * fs) + 16, dtype=torch.uint8, device="cuda")
        cfws.fill_splitmix(pay, 1)
        d_t = cfws.desc_to_device(desc)
        wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
        back = torch.empty(n * fs + 16 * n + 64, dtype=torch.uint8, device="cuda")
        idx = torch.from_numpy(offs.astype(np.int64)).cuda()
        dd = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        t1 = torch.zeros(1, dtype=torch.int64, device="cuda")
        t2 = torch.zeros(1, dtype=torch.int64, device="cuda")
        ws1 = cfws.workspace(n, wire.numel())
        ws2 = cfws.workspace(n, back.numel())
        gs = cfws.Graph.serialize(pay, d_t, wire, ws1, t1)
        gd = cfws.Graph.deserialize(wire, wtotal, idx, dd, st, back, ws2, t2)

        def eager():
            cfws.serialize(pay, d_t, wire, ws1, t1)
            cfws.deserialize(wire, wtotal, idx, back, dd, st, ws2, t2)

        def graph():
            gs.launch()
            gd.launch()

        for mode, fn in (("eager", eager), ("graph", graph)):
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            lat = []
            for _ in range(a.iters):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            torch.cuda.synchronize()
            pipe = (time.perf_counter() - t0) / a.iters
            back.zero_()
            fn()
            torch.cuda.synchronize()
            # deserialize lays payloads out at 16-byte-aligned offsets
            # (align 16): frame i's payload at i * round16(fs)
            a16 = W.round16(fs)
            ok = bool((st == 0).all()) and torch.equal(back[:n * a16].view(n, a16)[:, :fs],
                                                       pay[:n * fs].view(n, fs))
            print(json.dumps({"frames": n, "frame_size": fs, "mode": mode, "stream": a.stream,
                              "latency_us": round(statistics.median(lat) * 1e6, 1),
                              "pipelined_us": round(pipe * 1e6, 1),
                              "pipelined_GiBps": round(2 * n * fs / pipe / 2**30, 2),
                              "verified": ok}), flush=True)
        gs.close()
        gd.close()


if __name__ == "__main__":
    main()
