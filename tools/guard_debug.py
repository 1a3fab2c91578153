"""Diagnose test_gpu_guard's flush-start serialize mismatch: the seed-21
batch serialized with each arena in torch memory or in a guarded VMM
buffer (flush end / flush start), in a fresh process, diffs against the
oracle printed per placement."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402
import test_gpu_guard as G  # noqa: E402

cfws.init()
payload, desc = G._seed21_batch(21)
exp, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
_, total = W.wire_layout(desc)
bufs = []


def make(kind, n):
    if kind == "torch":
        t = torch.full((W.round16(n),), 0xEE, dtype=torch.uint8, device="cuda")
        return t
    b = G.GuardBuf(n, kind == "end")
    bufs.append(b)
    return b


def upload(b, a):
    if isinstance(b, torch.Tensor):
        b[:a.size].copy_(torch.from_numpy(a))
    else:
        b.upload(a)


def download(b, n):
    torch.cuda.synchronize()
    if isinstance(b, torch.Tensor):
        return b[:n].cpu().numpy()
    return b.download(n)


free_each = "--free" in sys.argv
args = [a for a in sys.argv[1:] if a != "--free"]
order = args or ["start:start", "torch:torch", "start:torch", "torch:start", "end:end",
                         "start:start"]
for spec in order:
    pk, wk = spec.split(":")
    pay = make(pk, payload.size)
    upload(pay, payload)
    back = download(pay, payload.size)
    up_ok = bool(np.array_equal(back, payload))
    wire = make(wk, total)
    tot = cfws.serialize(pay, cfws.desc_to_device(desc), wire)
    got = download(wire, total)
    bad = np.nonzero(got != exp)[0]
    info = {"payload": pk, "wire": wk, "payload_ptr_mod_2M": pay.data_ptr() % (2 << 20),
            "wire_ptr_mod_2M": wire.data_ptr() % (2 << 20), "upload_ok": up_ok,
            "total_ok": int(tot.item()) == total, "bad": int(bad.size)}
    if bad.size:
        info["first"] = [(int(i), int(got[i]), int(exp[i])) for i in bad[:12]]
        # the payload bytes those wire bytes should come from
        offs, _ = W.wire_layout(desc)
        i0 = int(bad[0])
        f = int(np.searchsorted(offs, i0, side="right") - 1)
        info["frame"] = {"f": f, "wire_off": int(offs[f]), "payload_off": int(desc["payload_off"][f]),
                         "size": int(desc["payload_size"][f]), "mask": int(desc["mask"][f])}
    print(info, flush=True)
    if free_each:           # unmap + free now: the next spec may reuse the address range
        torch.cuda.synchronize()
        for b in bufs:
            b.free()
        bufs.clear()
for b in bufs:
    b.free()
