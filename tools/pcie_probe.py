"""PCIe probe for the host-memory path: DMA copies of pinned host memory one
way and both ways at once. Prints one JSON line.

(Kernels must not dereference torch's pinned host pointers directly: a
first zero-copy attempt faulted the GPU -- torch's pinned allocations are
not guaranteed to be mapped at the same address for the device.)

usage: python tools/pcie_probe.py [MiB]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from coldforce_amd import cfws  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    cfws.init()
    h_a = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_b = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_a.fill_(7)
    d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {"bytes": n}

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_a, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_b.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    res["h2d_GBps"] = n / timed(h2d) / 1e9
    res["d2h_GBps"] = n / timed(d2h) / 1e9
    res["bidir_GBps_each"] = n / timed(both) / 1e9
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
