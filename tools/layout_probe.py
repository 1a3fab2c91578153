"""Does the arenas' relative placement in HBM move the streaming kernel's rate?

Config 2 (65,536 x 64 KiB) serialize and deserialize executes, timed with HIP
events, with the payload, wire and unmasked-copy arenas carved out of one
allocation at chosen offsets (and once as three separate allocations, the
bench's layout). Prints one JSON line per layout. Diagnostic only (DESIGN.md
section 3.4's send/receive asymmetry).

  python tools/layout_probe.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GIB = 1 << 30
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--orders", default="", help="e.g. SSSS,DDDD,SDSD: time each execute after another")
    ap.add_argument("--align", type=int, default=16, help="deserialize payload alignment (orders mode)")
    args = ap.parse_args()
    import torch
    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    cfws.init()
    dev = torch.device("cuda", 0)
    F, fs = args.frames, 65536
    desc_np, _ = shard.uniform_shard(F, fs, 2, 0, 1)
    offs, wire_total = W.wire_layout(desc_np)
    n = F * fs
    wn = W.round16(wire_total)
    desc_ser = cfws.desc_to_device(desc_np, dev)
    desc_de = torch.empty((F, 32), dtype=torch.uint8, device=dev)
    status = torch.empty(F, dtype=torch.int32, device=dev)
    index = torch.from_numpy(offs.astype("int64")).to(dev)
    tot_ser = torch.zeros(1, dtype=torch.int64, device=dev)
    tot_de = torch.zeros(1, dtype=torch.int64, device=dev)
    alg = 2 * n + (wire_total - n)

    def run(name, payload, wire, back):
        cfws.fill_splitmix(payload, 0x5EED0002, 0)
        ws_ser = cfws.workspace(F, wire.numel(), dev)
        ws_de = cfws.workspace(F, back.numel(), dev)
        cfws.serialize_plan(desc_ser, wire.numel(), tot_ser, ws_ser)
        cfws.serialize_execute(payload, desc_ser, wire, ws_ser)
        cfws.deserialize_plan(wire, wire_total, index, desc_de, status, back.numel(), tot_de, ws_de, align=16)
        cfws.deserialize_execute(wire, desc_de, status, back, ws_de)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ser, de = [], []
        for _ in range(args.reps):
            ev[0].record()
            cfws.serialize_execute(payload, desc_ser, wire, ws_ser)
            ev[1].record()
            ev[2].record()
            cfws.deserialize_execute(wire, desc_de, status, back, ws_de)
            ev[3].record()
            torch.cuda.synchronize()
            ser.append(ev[0].elapsed_time(ev[1]))
            de.append(ev[2].elapsed_time(ev[3]))
        ok = torch.equal(back[:n], payload[:n])
        ser.sort()
        de.sort()
        s_ms, d_ms = ser[len(ser) // 2], de[len(de) // 2]
        print(json.dumps({"layout": name, "ser_ms": round(s_ms, 4), "deser_ms": round(d_ms, 4),
                          "ser_TBps": round(alg / s_ms / 1e9, 3), "deser_TBps": round(alg / d_ms / 1e9, 3),
                          "payload_addr_mod_2m": payload.data_ptr() % (2 * MIB),
                          "wire_minus_payload": wire.data_ptr() - payload.data_ptr(),
                          "back_minus_wire": back.data_ptr() - wire.data_ptr(), "ok": ok}), flush=True)
        del ws_ser, ws_de

    # the bench's layout: three allocations
    payload = torch.empty(n, dtype=torch.uint8, device=dev)
    wire = torch.empty(wn, dtype=torch.uint8, device=dev)
    back = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    if args.orders:
        # each execute's time by what ran before it (same arenas)
        cfws.fill_splitmix(payload, 0x5EED0002, 0)
        ws_ser = cfws.workspace(F, wire.numel(), dev)
        ws_de = cfws.workspace(F, back.numel(), dev)
        cfws.serialize_plan(desc_ser, wire.numel(), tot_ser, ws_ser)
        cfws.serialize_execute(payload, desc_ser, wire, ws_ser)
        cfws.deserialize_plan(wire, wire_total, index, desc_de, status, back.numel(), tot_de, ws_de,
                              align=args.align)
        # T: serialize reading the unmasked copy D wrote; E: deserialize from a
        # second wire arena written once at setup and never again
        wire2 = torch.empty_like(wire)
        wire2.copy_(wire)
        back2 = torch.empty_like(back)
        ops = {"S": lambda: cfws.serialize_execute(payload, desc_ser, wire, ws_ser),
               "D": lambda: cfws.deserialize_execute(wire, desc_de, status, back, ws_de),
               "T": lambda: cfws.serialize_execute(back, desc_ser, wire, ws_ser),
               "E": lambda: cfws.deserialize_execute(wire2, desc_de, status, back2, ws_de),
               "C": lambda: back[:n].copy_(payload)}
        for seq in args.orders.split(","):
            times = {k: [] for k in range(len(seq))}
            for _ in range(args.reps):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(seq) + 1)]
                ev[0].record()
                for k, c in enumerate(seq):
                    ops[c]()
                    ev[k + 1].record()
                torch.cuda.synchronize()
                for k in range(len(seq)):
                    times[k].append(ev[k].elapsed_time(ev[k + 1]))
            out = []
            for k, c in enumerate(seq):
                t = sorted(times[k])[len(times[k]) // 2]
                out.append({"op": c, "ms": round(t, 4), "TBps": round(alg / t / 1e9, 3)})
            print(json.dumps({"order": seq, "align": args.align, "edge_split": os.environ.get("CFWS_EDGE_SPLIT", "0"),
                              "ops": out}), flush=True)
        return
    run("separate", payload, wire, back)
    run("separate_swapped_roles", back[:n], wire, payload[:n])   # payload from the third allocation
    del payload, wire, back
    torch.cuda.empty_cache()
    big = torch.empty(3 * 4 * GIB + 64 * MIB, dtype=torch.uint8, device=dev)
    slot = 4 * GIB + 8 * MIB
    for name, po, wo, bo in [
        ("carved", 0, slot, 2 * slot),
        ("wire_first", slot, 0, 2 * slot),
        ("wire+256", 0, slot + 256, 2 * slot),
        ("wire+4k", 0, slot + 4096, 2 * slot),
        ("wire+64k", 0, slot + 65536, 2 * slot),
        ("wire+1m", 0, slot + MIB, 2 * slot),
        ("payload+4k", 4096, slot, 2 * slot),
        ("back+4k", 0, slot, 2 * slot + 4096),
        ("back+64k", 0, slot, 2 * slot + 65536),
    ]:
        run(name, big[po:po + n], big[wo:wo + wn], big[bo:bo + n + 64])


if __name__ == "__main__":
    main()
