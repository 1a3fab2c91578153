"""PCIe probe for the host-memory path: DMA copies one way and both ways at
once, and kernels that read / write pinned host memory directly (zero-copy,
cfws_xor_mask on mapped host pointers). Prints one JSON line.

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
    # zero-copy kernels (mapped pinned host memory)
    L = cfws.lib()
    st = torch.cuda.current_stream().cuda_stream

    def k_h2d():
        assert L.cfws_xor_mask(h_a.data_ptr(), d_a.data_ptr(), n, 0x01020304, 0, st) == 0

    def k_d2h():
        assert L.cfws_xor_mask(d_a.data_ptr(), h_b.data_ptr(), n, 0x01020304, 0, st) == 0

    def k_h2h():
        assert L.cfws_xor_mask(h_a.data_ptr(), h_b.data_ptr(), n, 0x01020304, 0, st) == 0

    for name, fn in (("kernel_read_host_GBps", k_h2d), ("kernel_write_host_GBps", k_d2h),
                     ("kernel_host_to_host_GBps_each", k_h2h)):
        try:
            res[name] = n / timed(fn) / 1e9
        except Exception as e:  # noqa: BLE001
            res[name] = f"error: {e}"
    torch.cuda.synchronize()
    ok = bool((h_b[:4096].cpu() == (h_a[:4096] ^ torch.tensor([4, 3, 2, 1], dtype=torch.uint8).repeat(1024))).all())
    res["kernel_h2h_verified"] = ok
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
