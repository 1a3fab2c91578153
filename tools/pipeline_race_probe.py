"""Diagnostic: repeat the host pipeline's config-2-reduced serialize (1,024 x
64 KiB, 8 MiB chunks, depth 3, torch-pinned host arenas, SDMA D2H) and the
device batch serialize of the same frames, and report where any run's wire
differs from the oracle's: byte ranges, the chunk and frame they fall in.

  python tools/pipeline_race_probe.py [--reps 10] [--depth 3] [--chunk-mib 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ranges(bad):
    out, start, prev = [], None, None
    for b in bad:
        if start is None:
            start = prev = b
        elif b == prev + 1:
            prev = b
        else:
            out.append((start, prev + 1))
            start = prev = b
    if start is not None:
        out.append((start, prev + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--chunk-mib", type=int, default=8)
    ap.add_argument("--d2h", default="auto")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle as O
    from coldforce_amd import cfws
    from coldforce_amd import workloads as W
    cfws.init()
    n, fs = 1024, 65536
    desc = W.uniform_batch(n, fs, 2)
    payload = O.splitmix_words(0x5EED0002, 0, n * fs // 8).view(np.uint8)
    exp, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    offs, total = W.wire_layout(desc)
    payload_t = torch.zeros(n * fs, dtype=torch.uint8, pin_memory=True)
    payload_t.numpy()[:] = payload
    wire_t = torch.zeros(total, dtype=torch.uint8, pin_memory=True)
    wire = wire_t.numpy()
    chunk = args.chunk_mib << 20
    for rep in range(args.reps):
        wire[:] = 0xEE
        pl = cfws.Pipeline(chunk_bytes=chunk, max_frames=4096, depth=args.depth, d2h=args.d2h)
        tot = pl.serialize(payload_t.data_ptr(), desc.copy(), wire_t.data_ptr(), wire.size)
        pl.close()
        bad = np.nonzero(wire[:total] != exp)[0]
        rs = ranges(bad.tolist()) if bad.size < 2_000_000 else [(int(bad[0]), int(bad[-1]) + 1)]
        info = [{"lo": lo, "hi": hi, "frame": int(np.searchsorted(offs, lo, side="right") - 1),
                 "chunk_of_8MiB_payload": int((np.searchsorted(offs, lo, side="right") - 1) * fs // chunk),
                 "got_head": wire[lo:min(hi, lo + 8)].tolist(), "exp_head": exp[lo:min(hi, lo + 8)].tolist()}
                for lo, hi in rs[:20]]
        print(json.dumps({"rep": rep, "kind": "pipeline", "total": int(tot), "bad_bytes": int(bad.size),
                          "ranges": len(rs), "first": info}), flush=True)
    # the device batch path on the same frames
    pd = torch.from_numpy(payload).cuda()
    for rep in range(max(1, args.reps // 2)):
        w = torch.full((W.round16(total),), 0xEE, dtype=torch.uint8, device="cuda")
        cfws.serialize(pd, cfws.desc_to_device(desc), w)
        torch.cuda.synchronize()
        got = w[:total].cpu().numpy()
        bad = np.nonzero(got != exp)[0]
        print(json.dumps({"rep": rep, "kind": "device", "bad_bytes": int(bad.size),
                          "first": ranges(bad.tolist())[:5]}), flush=True)


if __name__ == "__main__":
    main()
