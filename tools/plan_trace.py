"""Per-block timeline of the single-pass plans (a CFWS_PLAN_TRACE build:
`make variant V=trace F=-DCFWS_PLAN_TRACE=1`, run with
CFWS_LIB=build/variants/libcfws_trace.so). For the bench's 16 M x 256 B
shape: the serialize plan (serialize_plan_single_kernel) and the fused
receive (deserialize_plan_single_kernel<true>), each launched a few times;
prints, per kernel, the spread of block start times and the per-block time
from the ticket to the end of the loads + scan, through the look-back, and
to the end, in microseconds (wall clock at 100 MHz)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
FS = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cfws.init()
L = cfws.lib()
L.cfws_debug_plan_trace.argtypes = [C.c_void_p, C.c_size_t]
desc = W.uniform_batch(F, FS, 2, opcode=cfws.OPCODE_BINARY)
offs, total = W.wire_layout(desc)
payload = torch.empty(F * FS, dtype=torch.uint8, device="cuda")
cfws.fill_splitmix(payload, 1)
d_t = cfws.desc_to_device(desc)
wire = torch.empty(W.round16(total), dtype=torch.uint8, device="cuda")
ws = cfws.workspace(F, wire.numel())
tot = torch.zeros(1, dtype=torch.int64, device="cuda")
idx = torch.from_numpy(offs.astype(np.int64)).cuda()
back = torch.empty(F * FS + 64, dtype=torch.uint8, device="cuda")
ws_de = cfws.workspace(F, back.numel())


def trace(nblocks):
    t = np.zeros((nblocks, 4), dtype=np.uint64)
    assert L.cfws_debug_plan_trace(t.ctypes.data, nblocks) == 0
    t = t.astype(np.int64)
    t -= t[:, 0].min()
    us = t / 100.0
    return {
        "blocks": nblocks,
        "kernel_us": round(float(us[:, 3].max()), 1),
        "start_spread_us": [round(float(np.percentile(us[:, 0], q)), 1) for q in (0, 50, 100)],
        "loads_scan_us_p50_p90": [round(float(np.percentile(us[:, 1] - us[:, 0], q)), 2) for q in (50, 90)],
        "lookback_us_p50_p90_max": [round(float(np.percentile(us[:, 2] - us[:, 1], q)), 2) for q in (50, 90, 100)],
        "after_us_p50_p90": [round(float(np.percentile(us[:, 3] - us[:, 2], q)), 2) for q in (50, 90)],
        "block_us_p50": round(float(np.percentile(us[:, 3] - us[:, 0], 50)), 2),
        "resident_p50": int(np.percentile([np.sum((us[:, 0] <= x) & (us[:, 3] > x)) for x in
                                            np.linspace(0, us[:, 3].max(), 64)], 50)),
    }


out = {"frames": F, "frame_size": FS}
for rep in range(3):
    cfws.serialize_plan(d_t, wire.numel(), tot, ws)
    torch.cuda.synchronize()
ITEMS = int(os.environ.get("TRACE_ITEMS", "8"))
SER_T = int(os.environ.get("TRACE_SER_THREADS", "512"))
FUSED_T = int(os.environ.get("TRACE_FUSED_THREADS", "1024"))
sb = (F + SER_T * ITEMS - 1) // (SER_T * ITEMS)
out["serialize_plan"] = trace(sb)
cfws.serialize_execute(payload, d_t, wire, ws)
torch.cuda.synchronize()
for rep in range(3):
    cfws.deserialize(wire, total, idx, back, ws_t=ws_de, align=16)
    torch.cuda.synchronize()
# the fused receive (frames averaging <= 512 B of wire), else the receive
# plan (deserialize_plan_single_kernel<false>, traced the same way)
DE_T = int(os.environ.get("TRACE_DE_THREADS", "256"))
if total // F <= 512:
    out["fused_receive"] = trace((F + 2 * FUSED_T - 1) // (2 * FUSED_T))
else:
    out["receive_plan"] = trace((F + 8 * DE_T - 1) // (8 * DE_T))
print(json.dumps(out))
