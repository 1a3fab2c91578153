"""Config-2 steps (serialize plan + execute, deserialize plan + execute)
with no timing events at all, for a kernel trace of the gaps between
launches (tools/lds_gap_probe.sh SET=4). Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    cfws.init()
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
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
        cfws.serialize_plan(desc_ser, wire.numel(), t1, ws_ser)
        cfws.serialize_execute(payload, desc_ser, wire, ws_ser)
        cfws.deserialize_plan(wire, wire_total, index, desc_de, status, back.numel(), t2, ws_de, align=16)
        cfws.deserialize_execute(wire, desc_de, status, back, ws_de)
    torch.cuda.synchronize()
    print("ok", bool(torch.equal(back[:F * fs], payload)))


if __name__ == "__main__":
    main()
