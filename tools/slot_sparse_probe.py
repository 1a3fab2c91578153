"""Slots much larger than their payloads: N frames of FS
bytes received into SLOT-byte slots, timed with HIP events -- the case where
the piece kernel runs one wave per frame (the batch's average frame bounds
its waves per frame). Prints one JSON line.
  python3 tools/slot_sparse_probe.py [N] [FS] [SLOT]"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from coldforce_amd import cfws  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fs = int(sys.argv[2]) if len(sys.argv) > 2 else 256
slot = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
cfws.init()
pay = torch.empty(n * fs + 16, dtype=torch.uint8, device="cuda")
cfws.fill_splitmix(pay, 7, 0)
keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda")
W = cfws.uniform_frame_bytes(fs, True)
wire = torch.empty(n * W + 64, dtype=torch.uint8, device="cuda")
cfws.serialize_uniform(pay, keys, n, fs, wire, opcode=cfws.OPCODE_BINARY, mask=True)
out = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
info = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
mm = torch.zeros(1, dtype=torch.int32, device="cuda")
for _ in range(3):
    cfws.deserialize_slots_uniform(wire, n * W, n, W, out, slot, info, mismatch_t=mm)
e0, e1 = cfws.TimingEvent(), cfws.TimingEvent()
reps = 10
e0.record()
for _ in range(reps):
    cfws.deserialize_slots_uniform(wire, n * W, n, W, out, slot, info, mismatch_t=mm)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
del e0, e1                                    # HIP events freed while the runtime is up
ok = int(mm.item()) == 0 and torch.equal(out.view(n, slot)[:, :fs].reshape(-1)[:1 << 20],
                                          pay[:n * fs].view(n, fs).reshape(-1)[:1 << 20])
print(json.dumps({"frames": n, "payload": fs, "slot": slot,
                  "kernel": cfws.lib().cfws_deserialize_slots_pass_kernel(n, n * W, slot).decode(),
                  "ms": round(ms, 4), "GBps": round((n * W + n * fs) / ms / 1e6, 1), "verified": ok}))
