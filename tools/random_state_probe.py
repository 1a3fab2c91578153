"""Diagnostic: does anything in a torch + HIP + libcfws process move glibc's
random() state behind the main thread's back? Between srandom(seed) and the
draws the main thread runs one kind of GPU / runtime work (or just sleeps);
the draws are then compared with the same seed's stream from a private
random_r state. A mismatch means some library call (on this thread or
another) consumed or reseeded the shared state in that window.

  python tools/random_state_probe.py [--reps 30]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch

    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    cfws.init()
    libc = C.CDLL(None)
    libc.random.restype = C.c_long
    dev = torch.device("cuda", 0)
    n = 64

    def expected(seed):
        return cfws.draw_mask_keys(n, seed=seed)          # private random_r stream

    def global_draw():
        k = np.zeros(n, np.uint32)
        cfws.lib().cfws_draw_mask_keys(n, None, k.ctypes.data)
        return k

    payload = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    desc = W.uniform_batch(16, 4096, 1)

    def work_small_batch():
        wire = torch.empty(1 << 17, dtype=torch.uint8, device=dev)
        cfws.serialize(payload, cfws.desc_to_device(desc, dev), wire)

    def work_sync():
        torch.cuda.synchronize()

    def work_pinned():
        t = torch.zeros(1 << 22, dtype=torch.uint8, pin_memory=True)
        del t

    def work_pipeline():
        p = cfws.Pipeline(chunk_bytes=1 << 20, max_frames=64, depth=2)
        p.close()

    def work_stream():
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.ones(1000, device=dev).sum()
        s.synchronize()

    def work_sleep():
        time.sleep(0.02)

    kinds = {"none": lambda: None, "sleep": work_sleep, "small_batch": work_small_batch,
             "sync": work_sync, "pinned": work_pinned, "pipeline": work_pipeline,
             "stream": work_stream}
    for name, fn in kinds.items():
        bad = 0
        for rep in range(args.reps):
            seed = 1000 + rep
            exp = expected(seed)
            libc.srandom(C.c_uint(seed))
            fn()
            got = global_draw()
            if not np.array_equal(got, exp):
                bad += 1
        print(json.dumps({"between_srandom_and_draws": name, "reps": args.reps, "mismatches": bad}),
              flush=True)


if __name__ == "__main__":
    main()
