"""Diagnostic: what the timing events cost a config-2 step. The bench
records four events per step (around both executes); a kernel trace showed
~6 us of idle GPU at each one, and none without events. Runs the bench's
step with no events, with torch.cuda.Event, and with hipEventCreateWithFlags
events of several flag sets, and prints ms per step (wall clock over the
timed steps, as bench.py) and the two executes' event times.

  python tools/event_gap_probe.py [--steps 20] [--warmup 3] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FLAGS = {"hip_default": 0x0, "hip_no_sys_fence": 0x20000000, "hip_release_device": 0x40000000}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    cfws.init()
    hip = C.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipEventDestroy.argtypes = [C.c_void_p]
    dev = torch.device("cuda", 0)
    F, fs = 65536, 65536
    desc_np, _ = shard.uniform_shard(F, fs, 2, 0, 1)
    offs, wire_total = W.wire_layout(desc_np)
    payload = torch.empty(F * fs, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, 0x5EED0002)
    wire = torch.empty(W.round16(wire_total), dtype=torch.uint8, device=dev)
    back = torch.empty(F * fs + 64, dtype=torch.uint8, device=dev)
    desc_ser = cfws.desc_to_device(desc_np, dev)
    desc_de = torch.empty((F, 32), dtype=torch.uint8, device=dev)
    status = torch.empty(F, dtype=torch.int32, device=dev)
    index = torch.from_numpy(offs.astype("int64")).to(dev)
    ws_ser = cfws.workspace(F, wire.numel(), dev)
    ws_de = cfws.workspace(F, back.numel(), dev)
    t1 = torch.zeros(1, dtype=torch.int64, device=dev)
    t2 = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step(rec):
        cfws.serialize_plan(desc_ser, wire.numel(), t1, ws_ser)
        rec(0)
        cfws.serialize_execute(payload, desc_ser, wire, ws_ser)
        rec(1)
        cfws.deserialize_plan(wire, wire_total, index, desc_de, status, back.numel(), t2, ws_de, align=16)
        rec(2)
        cfws.deserialize_execute(wire, desc_de, status, back, ws_de)
        rec(3)

    def run(mode):
        evs, elapsed = [], None
        if mode == "none":
            def make(k):
                return lambda i: None
        elif mode == "torch":
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(a.steps)]
            def make(k):
                return lambda i: evs[k][i].record()
        else:
            for _ in range(a.steps):
                row = []
                for _ in range(4):
                    e = C.c_void_p()
                    assert hip.hipEventCreateWithFlags(C.byref(e), FLAGS[mode]) == 0
                    row.append(e)
                evs.append(row)
            def make(k):
                return lambda i: hip.hipEventRecord(evs[k][i], C.c_void_p(stream))
        for _ in range(a.warmup):
            step(lambda i: None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(make(k))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        ser = de = None
        if mode == "torch":
            ser = sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps
            de = sum(e[2].elapsed_time(e[3]) for e in evs) / a.steps
        elif mode != "none":
            f = C.c_float()
            s1 = s2 = 0.0
            for row in evs:
                hip.hipEventElapsedTime(C.byref(f), row[0], row[1]); s1 += f.value
                hip.hipEventElapsedTime(C.byref(f), row[2], row[3]); s2 += f.value
                for e in row:
                    hip.hipEventDestroy(e)
            ser, de = s1 / a.steps, s2 / a.steps
        return ms, ser, de

    for rep in range(a.reps):
        for mode in ["none", "torch"] + list(FLAGS):
            ms, ser, de = run(mode)
            print(json.dumps({"rep": rep, "events": mode, "ms_per_step": round(ms, 4),
                              "GiBps": round(2 * F * fs * 1e3 / ms / (1 << 30), 1),
                              "ser_ms": ser and round(ser, 4), "de_ms": de and round(de, 4)}), flush=True)


if __name__ == "__main__":
    main()
