"""Diagnostic: the host-pipeline serialize paths of tests/test_gpu_pipeline.py
(torch-pinned host arenas, SDMA D2H), repeated in one process, each result
checked against the oracle; a mismatch is reported with where it lies
(bytes, frames, chunk). Used to size a rare mismatch seen once in a full GPU
suite run. The library under test: CFWS_LIB (default the in-tree build).

  python tools/pipeline_stress.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle as O
    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    cfws.init()

    def pinned(n):
        t = torch.zeros(max(n, 16), dtype=torch.uint8, pin_memory=True)
        return t, t.numpy()

    def report(kind, rep, got, exp, offs):
        bad = np.nonzero(got != exp)[0]
        fr = np.unique(np.searchsorted(offs, bad, side="right") - 1) if bad.size else np.zeros(0, int)
        print(json.dumps({"rep": rep, "kind": kind, "bad_bytes": int(bad.size),
                          "first": bad[:6].tolist(), "frames": fr[:12].tolist(), "n_frames_bad": int(fr.size)}),
              flush=True)
        return bad.size

    # the random-mix case (chunk 69,632, depth 3)
    rng = random.Random(69632 + 3)
    payload_t, payload = pinned(3 << 20)
    payload[:] = O.fill_splitmix(payload.size, 77, 0)
    n = 3000
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    off = 0
    for i in range(n):
        sz = rng.choice([0, 1, 5, 125, 126, 1000, 4000, 20000, 65535, 65536, 65537 - 40000])
        if rng.random() < 0.5:
            off = rng.randrange(0, payload.size - sz)
        d[i] = (off, 0, sz, rng.getrandbits(32), rng.random() < .7, rng.choice([0, 1, 2, 9]),
                rng.random() < .6, 0)
        off = min(off + sz, payload.size - 70000)
    exp_mix, exp_d = O.serialize_batch(payload, d.view(O.DESC_DTYPE))
    # config 2 reduced (1,024 x 64 KiB, chunk 8 MiB, depth 3)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_digests.json")))[0]
    n2, fs = g["n_frames"], g["frame_size"]
    desc2 = W.uniform_batch(n2, fs, g["key_seed"])
    p2_t, p2 = pinned(n2 * fs)
    p2[:] = O.splitmix_words(g["payload_seed"], 0, n2 * fs // 8).view(np.uint8)
    exp2, _ = O.serialize_batch(p2, desc2.view(O.DESC_DTYPE))
    offs2, _ = W.wire_layout(desc2)
    bad_total = 0
    for rep in range(args.reps):
        wire_t, wire = pinned(len(exp_mix) + 64)
        p = cfws.Pipeline(chunk_bytes=69632, max_frames=512, depth=3)
        dd = d.copy()
        tot = p.serialize(payload_t.data_ptr(), dd, wire_t.data_ptr(), wire.size)
        p.close()
        bad_total += report("mix", rep, wire[:tot], exp_mix, exp_d["wire_off"])
        w2_t, w2 = pinned(g["wire_len"])
        p = cfws.Pipeline(chunk_bytes=8 << 20, max_frames=4096, depth=3)
        tot2 = p.serialize(p2_t.data_ptr(), desc2.copy(), w2_t.data_ptr(), w2.size)
        p.close()
        bad_total += report("config2", rep, w2[:tot2], exp2, offs2)
        del wire_t, w2_t
    print(json.dumps({"summary": True, "reps": args.reps, "bad_bytes_total": int(bad_total),
                      "lib": os.environ.get("CFWS_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()
