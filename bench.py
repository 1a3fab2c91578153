#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: device-resident WebSocket payload
mask/unmask GiB/s on 64 KiB binary frames, one process per MI355X.

Workload (BASELINE.json configs[1]): per GPU a batch
of 65,536 binary frames x 64 KiB payload (4 GiB), client-mask then
server-unmask, device resident. One step =
  cfws_serialize_plan + cfws_serialize_execute    (co_ws_frame_serialize x 65,536,
                                                   mask = true: header + XOR mask)
  cfws_deserialize_plan + cfws_deserialize_execute (co_ws_frame_deserialize at every
                                                   frame start: header parse + copy
                                                   + XOR unmask)
value = payload bytes processed by both ops on all ranks / wall time of the
K timed steps (max over ranks), in GiB/s (2^30). With N GPUs each rank owns
its own 65,536-frame shard of one global batch (weak scaling, no collective
on the data path; the only collectives are the timing barrier and max, and
a gather of each rank's timings for the line's per_gpu rows). The executes
are timed with HIP events on the stream they run on (cfws.TimingEvent:
created without the system-scope fence, which torch.cuda.Event records and
which left ~6 us of idle GPU in the stream at each record).

Usage: python bench.py [--gpus N --steps K --warmup W]
         (N > 1: this process starts N workers itself, one per GPU, and makes
          no GPU call; spawn_ranks)
       torchrun --nproc-per-node N bench.py --gpus N ...   (the same run under torchrun)
The ranks' bookkeeping collectives run over gloo (RCCL is never initialised).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GIB = float(1 << 30)
METRIC = "WS payload mask/unmask GiB/s device-resident, 64KiB frames, 1/2/4/8 GPUs"
PAYLOAD_SEED = 0x5EED0002
KEY_SEED = 2
CONFIG4 = dict(frames_total=8 << 20, shards=8, payload_seed=0x5EED0004, key_seed=4)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames", type=int, default=65536, help="frames per GPU")
    ap.add_argument("--frame-size", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU time of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: only the multi-rank launch and bookkeeping (CPU test)")
    ap.add_argument("--recv-slots", action="store_true",
                    help="config2: receive into fixed payload slots of frame-size bytes "
                         "(cfws_deserialize_slots) instead of the packed layout")
    ap.add_argument("--recv-scatter", action="store_true",
                    help="config2: receive each frame to its own offset, the slots in a "
                         "shuffled order (cfws_deserialize_scatter)")
    ap.add_argument("--send", choices=["batch", "uniform"], default="batch",
                    help="config2: the send through cfws_serialize_batch (descriptor table + "
                         "plan + execute) or cfws_serialize_uniform (payload + one key per "
                         "frame, no plan: the compact form of a uniform batch)")
    ap.add_argument("--recv-info", action="store_true",
                    help="with --recv-slots / --recv-scatter: the compact 8-byte per-frame output "
                         "(cfws_deserialize_slots_info / _scatter_info) instead of descriptors + statuses")
    ap.add_argument("--recv-uniform", action="store_true",
                    help="config2: the slot receive of a uniform stream, frame i at i x its wire "
                         "bytes with no index (cfws_deserialize_slots_uniform, compact output and a "
                         "mismatch count); implies --recv-slots --recv-info")
    ap.add_argument("--keys", type=int, default=1 << 20, help="accept workload: client keys per GPU")
    ap.add_argument("--connections", type=int, default=16384, help="index workload: connections")
    ap.add_argument("--index-mib", type=int, default=1024, help="index workload: receive-buffer MiB")
    ap.add_argument("--workload", choices=["config2", "config3", "config4", "config5", "split", "accept",
                                           "index"],
                    default="config2",
                    help="config2: uniform 64 KiB frames (the metric's config); config3: Zipf "
                         "64 B-1 MiB messages in 1-8 continuation fragments, reassembled; "
                         "config4: the 8 M x 64 KiB batch cut in 8 shards, rank r runs shard r "
                         "(1,048,576 frames = 64 GiB per GPU); "
                         "config5: WebSocket over HTTP/2 DATA frames (--frame-size, default "
                         "16376); split: config 2 through the split ops (encode_headers + "
                         "mask_batch, parse_headers + unmask_batch); accept: handshake accept "
                         "keys for a connection storm (--keys); index: the receive loop's frame "
                         "walk over many connections (--connections, --index-mib)")
    return ap.parse_args()


def host_cpus() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_limit():
    """The job's cgroup CPU quota ("max" or "<quota> <period>"), if any: on
    a shared box nproc can exceed the CPU time the job is given."""
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            continue
    return None


def effective_cpus() -> int:
    """The CPUs this job may use at once: nproc, or fewer when the cgroup's
    quota (cpu.max) grants fewer (the GPU box: 256 CPUs visible, a 16-CPU
    quota). Threads beyond it only queue."""
    n = host_cpus()
    q = cgroup_cpu_limit()
    try:
        quota, period = q.split()[:2]
        if quota != "max" and int(period) > 0:
            n = max(1, min(n, int(quota) // int(period)))
    except (AttributeError, ValueError):
        pass
    return n


def cpu_baseline(frame_size: int, seconds: float):
    """Reference codec (oracle/_ref, compiled from coldforce's own sources at
    -O2) when it was built, else the clean-room port; timed on this host
    (SURVEY.md 8(d)): a sweep over 1/8/16/32/64 threads up to the CPUs the
    job's cgroup grants (effective_cpus) plus nproc, at -O2, and the
    as-shipped -O0 at 1 and the best thread count. `value` is the fastest
    point of the sweep, `cores` its thread count.

    Only the combined rate (mask + unmask payload bytes over the time of
    both) is reported. The per-frame loop alternates a mask phase (bound by
    glibc's random() lock) and an unmask phase of a few ms each, so under a
    CPU quota a phase timed alone can run on time the other phase left
    unspent, and a split rate would overstate what the host sustains."""
    import oracle
    kind = "reference" if oracle.ref_lib("O2") is not None else "port"
    cpus = host_cpus()
    eff = effective_cpus()

    def frames_for(threads):
        return max(256, 64 * threads)

    def rate(k, threads, target_s):
        """(payload bytes of one direction, seconds of mask + unmask, iters)."""
        n = frames_for(threads)
        oracle.cpu_bench(n, frame_size, threads, 1, k)          # first touch of the heaps
        m1, u1 = oracle.cpu_bench(n, frame_size, threads, 2, k)
        it = max(1, int(math.ceil(2 * target_s / max(m1 + u1, 1e-3))))
        if it > 1:
            m1, u1 = oracle.cpu_bench(n, frame_size, threads, it, k)
        return n * frame_size * it, m1 + u1, it

    # the sweep first (short samples), then the main sample on the thread
    # count that ran fastest: on a shared box the job's cgroup can grant far
    # fewer CPUs than nproc shows (cpu.max), and the reference's key draws
    # serialise on glibc's random() lock, so nproc threads can be the
    # slowest choice; every point is reported
    sweep = []
    for t in sorted({1, 8, 16, 32, 64, eff, cpus}):
        if t > cpus or (t > eff and t != cpus):
            continue
        p, sec, _ = rate(kind, t, 1.5)
        sweep.append({"threads": t, "gibs": round(2 * p / sec / GIB, 3)})
    best = max(sweep, key=lambda r: r["gibs"])["threads"]
    payload, sec, iters = rate(kind, best, seconds)
    as_shipped = {}
    if kind == "reference":
        for t in sorted({1, best}):
            p, s0, _ = rate("reference_O0", t, 1.5)
            as_shipped[str(t)] = round(2 * p / s0 / GIB, 3)
    p, s1, _ = rate("port", 1, 1.5)
    n = frames_for(best)
    return {
        "value": round(2 * payload / sec / GIB, 3),
        "unit": "GiB/s",
        "cores": best,
        "kind": kind,
        "sample": (f"{n} x {size_label(frame_size)} binary frames x {iters} iters, per-frame "
                   f"co_ws_frame_serialize(mask) + co_ws_frame_deserialize"
                   f"{' (reference -O2, oracle/_ref)' if kind == 'reference' else ' (port, -O2)'},"
                   f" {best} threads (the fastest of the sweep; cgroup grants {eff} of nproc = "
                   f"{cpus}), each on a contiguous frame range; mask and unmask timed as one "
                   f"combined rate"),
        "seconds": round(sec, 2),
        "nproc": cpus,
        "effective_cpus": eff,
        "scaling_O2": sweep,
        "as_shipped_O0": as_shipped,
        "port_O2_1_thread": round(2 * p / s1 / GIB, 3),
        "cgroup_cpu_max": cgroup_cpu_limit(),
    }


def cpu_baseline_h2(frame_size: int, max_frame: int, seconds: float):
    """Config 5 on this host through the reference compiled in place
    (oracle/_ref: co_ws_frame.c + co_http2_frame.c + the send split of
    co_http2_stream.c:933-1013 and the pooling of :550-608, per WS frame; see
    oracle/cpu_bench.c ref_h2_cpu_bench), swept like cpu_baseline over thread
    counts up to the cgroup's grant; the main sample on the fastest. None
    when oracle/_ref was not built."""
    import oracle
    if oracle.ref_lib("O2") is None:
        return None
    cpus, eff = host_cpus(), effective_cpus()

    def rate(threads, target_s):
        n = max(256, 64 * threads)
        oracle.cpu_h2_bench(n, frame_size, max_frame, threads, 1)
        s1, r1 = oracle.cpu_h2_bench(n, frame_size, max_frame, threads, 2)
        it = max(1, int(math.ceil(2 * target_s / max(s1 + r1, 1e-3))))
        if it > 1:
            s1, r1 = oracle.cpu_h2_bench(n, frame_size, max_frame, threads, it)
        return n * frame_size * it, s1, r1, it, n

    sweep = []
    for t in sorted({1, 8, 16, 32, 64, eff, cpus}):
        if t > cpus or (t > eff and t != cpus):
            continue
        p, s1, r1, _, _ = rate(t, 1.5)
        sweep.append({"threads": t, "gibs": round(2 * p / (s1 + r1) / GIB, 3)})
    best = max(sweep, key=lambda r: r["gibs"])["threads"]
    p, s1, r1, iters, n = rate(best, seconds)
    return {
        "value": round(2 * p / (s1 + r1) / GIB, 3),
        "unit": "GiB/s",
        "cores": best,
        "kind": "reference",
        "sample": (f"{n} x {size_label(frame_size)} binary frames x {iters} iters, per WS frame "
                   f"co_ws_frame_serialize(mask) + DATA frames of <= {max_frame} B through "
                   f"co_http2_frame.c (send), co_http2_frame_deserialize + pooling + "
                   f"co_ws_frame_deserialize (receive); reference -O2 (oracle/_ref), {best} threads "
                   f"(the fastest of the sweep; cgroup grants {eff} of nproc = {cpus}); send and "
                   f"receive timed as one combined rate"),
        "send_GiBps": round(p / s1 / GIB, 3),
        "receive_GiBps": round(p / r1 / GIB, 3),
        "seconds": round(s1 + r1, 2),
        "nproc": cpus,
        "effective_cpus": eff,
        "scaling_O2": sweep,
    }


def size_label(n: int) -> str:
    """64 KiB, 1 KiB, 256 B, 16376 B: the frame size as the workload names it."""
    return f"{n // 1024} KiB" if n >= 1024 and n % 1024 == 0 else f"{n} B"


def load_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary taken
    on exactly this workload (profiles/pmc_traffic*.json, written by
    tools/pmc_summary.py with its "workload" key), or None when no PMC pass
    has been run on it."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json"))):
        try:
            with open(path) as f:
                data = json.load(f)
        except (OSError, ValueError):
            continue
        if data.get("workload") == workload:
            return data.get(kernel, {}).get("hbm_bytes_per_launch")
    return None


def bench_h2(args, rank, world, dev):
    """Config 5, device resident: WS frames -> HTTP/2 DATA frames (send) and
    DATA frames -> pooled messages -> payloads (receive), per step."""
    import numpy as np
    import torch

    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    F = args.frames
    fs = args.frame_size if args.frame_size != 65536 or "--frame-size" in sys.argv else 16376
    S = cfws.H2_DEFAULT_MAX_FRAME_SIZE
    desc_np, byte_base = shard.uniform_shard(F, fs, 5, rank, world)
    payload = torch.empty(W.round16(F * fs) + 16, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, 0x5EED0005, byte_base)
    offs, wtotal = W.wire_layout(desc_np)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device=dev)
    h2 = torch.empty(cfws.h2_wrapped_bound(wire.numel(), F, S), dtype=torch.uint8, device=dev)
    d_t = cfws.desc_to_device(desc_np, dev)
    ws_s = torch.empty(cfws.lib().cfws_h2_serialize_workspace_size(F, wire.numel(), h2.numel(), S),
                       dtype=torch.uint8, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    cfws.h2_serialize(payload, d_t, wire, h2, 1, S, ws_s, tot)
    torch.cuda.synchronize()
    h2_total = int(tot.item())
    Wf = int(offs[1] - offs[0]) if F > 1 else wtotal
    k = -(-Wf // S)
    per = np.arange(F, dtype=np.uint64) * np.uint64(Wf + 9 * k)
    starts = (per[:, None] + (np.arange(k, dtype=np.uint64) * np.uint64(S + 9))[None, :]).reshape(-1)
    idx_t = torch.from_numpy(starts.astype(np.int64)).to(dev)
    pool = torch.empty(h2_total, dtype=torch.uint8, device=dev)
    back = torch.empty(F * fs + 64, dtype=torch.uint8, device=dev)
    ws_d = torch.empty(cfws.lib().cfws_h2_deserialize_workspace_size(len(starts), pool.numel(),
                                                                      back.numel()),
                       dtype=torch.uint8, device=dev)

    def step(ev=None):
        # ev: the streaming pass of each call timed by events on its stream
        # (cfws_time_next_pass: recorded right around the xform_kernel launch)
        if ev:
            cfws.time_next_pass(ev[0], ev[1])
        cfws.h2_serialize(payload, d_t, wire, h2, 1, S, ws_s, tot)
        if ev:
            cfws.time_next_pass(ev[2], ev[3])
        return cfws.h2_deserialize(h2, h2_total, idx_t, pool, back, S, align=1, ws_t=ws_d)

    for _ in range(args.warmup):
        step()
    events = [[cfws.TimingEvent() for _ in range(4)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        st, md, ms, ptot, m = step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local, dev)
    send_each = [e[0].elapsed_time(e[1]) for e in events]
    recv_each = [e[2].elapsed_time(e[3]) for e in events]
    send_ms, recv_ms = sum(send_each) / args.steps, sum(recv_each) / args.steps
    del events
    # algorithmic bytes per pass: read the payload n, write n plus every
    # header (WS + DATA) on the send; the receive reads what the send wrote
    # past the headers and writes n -- 2n + headers either way
    alg = F * fs + h2_total
    kern = {"h2_serialize_pass": {"kernel": "xform_kernel<3>", "ms": round(send_ms, 4),
                                  "median_ms": round(statistics.median(send_each), 4),
                                  "GBps": round(alg / (send_ms * 1e-3) / 1e9, 1)},
            "h2_deserialize_pass": {"kernel": "xform_kernel<1>", "ms": round(recv_ms, 4),
                                    "median_ms": round(statistics.median(recv_each), 4),
                                    "GBps": round(alg / (recv_ms * 1e-3) / 1e9, 1)}}
    dom = "h2_serialize_pass" if send_ms >= recv_ms else "h2_deserialize_pass"
    dom_ms = max(send_ms, recv_ms)
    achieved = alg / (dom_ms * 1e-3) / 1e9
    rows = shard.gather_floats([local, F * fs], dev)
    ok = (m == F and int(ptot.item()) == F * fs and bool((st == 0).all()) and bool((ms == 0).all())
          and torch.equal(back[:F * fs], payload[:F * fs]))
    ok = shard.sum_over_ranks(1.0 if ok else 0.0, dev) == world
    line = {"metric": "WS-over-HTTP/2 payload GiB/s device-resident (config 5)",
            "value": round(2.0 * F * fs * world * args.steps / elapsed / GIB, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "dtype": "u8",
            "config": {"workload": f"config5: {F} binary frames x {fs} B per GPU, client-mask + "
                                   f"HTTP/2 DATA wrap (max frame {S}), then DATA unwrap + pool + "
                                   f"server-unmask", "h2_bytes_per_gpu": h2_total,
                       "data_frames_per_gpu": len(starts)},
            "roofline": {"bound": "hbm", "kernel": kern[dom]["kernel"], "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(kern[dom]["kernel"], f"config5:{F}x{fs}"),
                         "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(dom_ms, 4)},
            "kernels": kern,
            "note": "one fused streaming pass per direction: WS frames straight into DATA frames (send), WS payload slices straight out of DATA frames (receive)",
            "per_gpu": per_gpu_rows(rows, args.steps), "verified": ok}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_h2(fs, S, args.cpu_seconds)
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


def bench_split(args, rank, world, dev):
    """Config 2 through the split ops of include/cfws.h: cfws_encode_headers
    + cfws_mask_batch_packed (send), cfws_parse_headers + cfws_unmask_batch
    (receive), per step; wire offsets laid out by the host."""
    import numpy as np
    import torch

    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    F, fs = args.frames, args.frame_size
    desc_np, byte_base = shard.uniform_shard(F, fs, KEY_SEED, rank, world)
    offs, wire_total = W.wire_layout(desc_np)
    desc_np["wire_off"] = offs
    payload = torch.empty(F * fs, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, PAYLOAD_SEED, byte_base)
    wire = torch.empty(W.round16(wire_total), dtype=torch.uint8, device=dev)
    back = torch.empty(F * fs, dtype=torch.uint8, device=dev)
    d_t = cfws.desc_to_device(desc_np, dev)
    idx = torch.from_numpy(offs.astype(np.int64)).to(dev)
    pd_t = torch.empty((F, 32), dtype=torch.uint8, device=dev)
    st_t = torch.empty(F, dtype=torch.int32, device=dev)
    # the receive side's payload layout: the frame index x frame size
    pay_off = torch.from_numpy((np.arange(F, dtype=np.uint64) * np.uint64(fs)).view(np.int64)).to(dev)

    # cfws_mask_batch_packed (the frames are packed back to back);
    # CFWS_BENCH_SPLIT_PACKED=0: cfws_mask_batch (A/B)
    packed = os.environ.get("CFWS_BENCH_SPLIT_PACKED", "1") != "0"

    def step():
        cfws.encode_headers(d_t, wire)
        cfws.mask_batch(payload, d_t, wire, fs, packed=packed)   # the frames are packed back to back
        cfws.parse_headers(wire, wire_total, idx, pd_t, st_t)
        pd_t.view(torch.int64)[:, 0] = pay_off
        cfws.unmask_batch(wire, pd_t, st_t, back, fs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local, dev)
    rows = shard.gather_floats([local, F * fs], dev)
    ok = bool((st_t == 0).all()) and torch.equal(back, payload)
    line = {"metric": "WS payload mask/unmask GiB/s device-resident, split ops (config 2 layout)",
            "value": round(2.0 * F * fs * world * args.steps / elapsed / GIB, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "config": {"workload": f"split: {F} binary frames x {fs} B per GPU: encode_headers + "
                                   f"mask_batch_packed, then parse_headers + unmask_batch"},
            "per_gpu": per_gpu_rows(rows, args.steps), "verified": ok}
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9     # lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes/clk x 2.4 GHz


def load_pmc(name: str, key: str):
    """A per-launch counter value from a committed PMC summary (profiles/)."""
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def bench_accept(args, rank, world, dev):
    """Sec-WebSocket-Accept for a connection storm
    (co_ws_create_base64_accept_key, co_ws_http_extension.c:26-57) -- one
    cfws_ws_accept_keys_batch over N client keys (24-character base64 of 16
    random bytes, RFC 6455 4.1) per step, device resident. Checked against the
    oracle on a sample; the CPU baseline runs the reference's co_sha1.c +
    co_base64.c (oracle/_ref) on the host's threads."""
    import base64
    import random

    import numpy as np
    import torch

    import oracle as O
    from coldforce_amd import cfws, shard
    N = args.keys
    rng = random.Random(0x5EED0006 + rank)
    keys = [base64.b64encode(rng.randbytes(16)) for _ in range(N)]
    raw = np.frombuffer(b"".join(keys), np.uint8).copy()
    off = np.zeros(N + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(k) for k in keys])
    d_keys = torch.from_numpy(raw).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    out = torch.zeros(N * cfws.WS_ACCEPT_SLOT, dtype=torch.uint8, device=dev)

    def step():
        cfws._check(cfws.lib().cfws_ws_accept_keys_batch(cfws._p(d_keys), cfws._p(d_off), N,
                                                         cfws._p(out), cfws._stream(None)),
                    "cfws_ws_accept_keys_batch")

    for _ in range(args.warmup):
        step()
    ev = [[cfws.TimingEvent() for _ in range(2)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        step()
        ev[k][1].record()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local, dev)
    kms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    del ev                                   # HIP events freed while the runtime is up
    h = out.view(N, cfws.WS_ACCEPT_SLOT)
    sample = list(range(0, N, max(1, N // 4096)))
    got = h[sample, :28].cpu().numpy()
    ok = all(bytes(got[j]).decode() == O.ws_accept_key(keys[i]) for j, i in enumerate(sample))
    ok = shard.sum_over_ranks(1.0 if ok else 0.0, dev) == world
    # VALU lane-ops per key from the committed PMC pass (SQ_INSTS_VALU x 64 /
    # keys, measured at 1,048,576 keys; per key, so it scales with --keys)
    per_key = load_pmc("pmc_accept.json", "valu_instructions_per_key")
    achieved = per_key * N / (kms * 1e-3) if per_key else None
    line = {"metric": "WS handshake Sec-WebSocket-Accept keys/s (SHA-1 + base64), device resident",
            "value": round(N * world * args.steps / elapsed, 1), "unit": "keys/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "dtype": "u32", "data": "synthetic (24-char base64 client keys)",
            "config": {"workload": f"accept: {N} client keys per GPU, one accept key per thread"},
            "roofline": {"bound": "valu", "kernel": "ws_accept_kernel", "avg_launch_ms": round(kms, 4),
                         "achieved": round(achieved / 1e12, 2) if achieved else None,
                         "peak": round(VALU_PEAK_OPS / 1e12, 1), "unit": "T lane-ops/s",
                         "frac": round(achieved / VALU_PEAK_OPS, 4) if achieved else None,
                         "valu_lane_ops_per_launch": per_key * N if per_key else None},
            "verified": ok}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        kind = "reference" if O.ref_lib("O2") is not None else "port"
        threads = effective_cpus()
        n = min(N, 262144)
        t1 = O.cpu_accept_bench(raw, off[:n + 1].astype(np.uint64), threads, 1, kind)
        iters = max(1, int(math.ceil(args.cpu_seconds / max(t1, 1e-3))))
        t = O.cpu_accept_bench(raw, off[:n + 1].astype(np.uint64), threads, iters, kind)
        line["cpu_baseline"] = {"value": round(n * iters / t, 1), "unit": "keys/s", "cores": threads,
                                "nproc": host_cpus(), "cgroup_cpu_max": cgroup_cpu_limit(),
                                "kind": kind, "sample": f"{n} keys x {iters} iters, one "
                                f"co_sha1 + co_base64_encode per key, {threads} threads",
                                "seconds": round(t, 2)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


def bench_index(args, rank, world, dev):
    """the receive loop's frame walk
    (co_ws_server.c:107-169) for many connections at once
    (cfws_index_frames_batch, one thread per connection), device resident.
    A server tick: args.connections receive buffers in one arena, each
    holding a run of client-masked 1 KiB TEXT frames (config 1's frame) and
    a cut last frame (MORE_DATA), args.index_mib MiB in all. Checked against
    the oracle's walk on a sample of connections; the CPU baseline is that
    walk on the host's threads over every connection."""
    import numpy as np
    import torch

    import oracle as O
    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W
    fs = 1024
    F = (args.index_mib << 20) // (fs + 8)
    desc = W.uniform_batch(F, fs, 1 + rank, opcode=cfws.OPCODE_TEXT)
    payload = torch.empty(F * fs + 16, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, 0x5EED0001 + rank, 0)
    offs, wtotal = W.wire_layout(desc)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device=dev)
    cfws.serialize(payload, cfws.desc_to_device(desc, dev), wire)
    torch.cuda.synchronize()
    C_ = args.connections
    rng = np.random.default_rng(17 + rank)
    first_frame = (np.arange(C_ + 1, dtype=np.int64) * F) // C_
    fstarts = np.concatenate([offs.astype(np.int64), [wtotal]])
    begin_np = fstarts[first_frame[:-1]]
    # each buffer ends inside its last frame (a partial read), or whole
    cut = rng.integers(0, fs + 8, C_)
    end_np = np.maximum(begin_np, fstarts[first_frame[1:]] - cut)
    d_begin = torch.from_numpy(begin_np).to(dev)
    d_end = torch.from_numpy(end_np).to(dev)
    starts_t = torch.empty(F + C_, dtype=torch.int64, device=dev)     # every frame start fits
    ws_t = torch.empty(cfws.lib().cfws_index_workspace_size(C_), dtype=torch.uint8, device=dev)
    first = torch.empty(C_, dtype=torch.int64, device=dev)
    consumed = torch.empty(C_, dtype=torch.int64, device=dev)
    stop = torch.empty(C_, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        cfws._check(cfws.lib().cfws_index_frames_batch(
            cfws._p(wire), cfws._p(d_begin), cfws._p(d_end), C_, cfws.DEFAULT_MAX_PAYLOAD,
            cfws._p(starts_t), starts_t.numel(), cfws._p(first), cfws._p(consumed), cfws._p(stop),
            cfws._p(total), cfws._p(ws_t), ws_t.numel(), cfws._stream(None)), "cfws_index_frames_batch")

    for _ in range(args.warmup):
        step()
    ev = [[cfws.TimingEvent() for _ in range(2)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        step()
        ev[k][1].record()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local, dev)
    kms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    del ev                                   # HIP events freed while the runtime is up
    n_frames = int(total.item())
    host_wire = wire[:wtotal].cpu().numpy()
    st_h, first_h = starts_t.cpu().numpy(), first.cpu().numpy()
    con_h, stop_h = consumed.cpu().numpy(), stop.cpu().numpy()
    ok = True
    for c in range(0, C_, max(1, C_ // 256)):
        e_st, e_con, e_stop = O.index_stream(host_wire, int(begin_np[c]), int(end_np[c]))
        ok &= bool(np.array_equal(st_h[first_h[c]:first_h[c] + len(e_st)].astype(np.uint64), e_st)
                   and con_h[c] == e_con and stop_h[c] == e_stop)
    ok = shard.sum_over_ranks(1.0 if ok else 0.0, dev) == world
    hops = n_frames / C_
    line = {"metric": "WS receive-buffer frame indexing frames/s, many connections, device resident",
            "value": round(n_frames * world * args.steps / elapsed, 1), "unit": "frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "dtype": "u8",
            "data": "synthetic (client-masked 1 KiB TEXT frames, buffers cut inside their last frame)",
            "config": {"workload": f"index: {C_} connections x {hops:.1f} frames, "
                                   f"{args.index_mib} MiB of receive buffers",
                       "wire_bytes": int(wtotal), "frames": n_frames, "connections": C_},
            "roofline": {"bound": "latency", "avg_launch_ms": round(kms, 4),
                         "note": "each connection is one walk, a chain of dependent header "
                                 "reads that keeps its first 64 starts in the workspace; after "
                                 "the scan of the counts, index_place copies them to their "
                                 "places and index_rest walks on for connections longer than "
                                 "64 frames. The launch is bounded by hop latency x chain "
                                 "length, not HBM bytes",
                         "ns_per_hop": round(kms * 1e6 / max(hops, 1e-9), 1)},
            "verified": ok}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = effective_cpus()
        ub = (begin_np.astype(np.uint64), end_np.astype(np.uint64))
        t1, _ = O.cpu_index_bench(host_wire, ub[0], ub[1], 4096, threads)
        reps = max(1, int(math.ceil(args.cpu_seconds / max(t1, 1e-3))))
        t, f = 0.0, 0
        for _ in range(reps):
            ti, fi = O.cpu_index_bench(host_wire, ub[0], ub[1], 4096, threads)
            t += ti
            f += fi
        line["cpu_baseline"] = {"value": round(f / t, 1), "unit": "frames/s", "cores": threads,
                                "nproc": host_cpus(), "cgroup_cpu_max": cgroup_cpu_limit(),
                                "kind": "port", "sample": f"every connection x {reps}, the receive "
                                f"loop's walk (orc_index_stream) over host memory, {threads} threads",
                                "seconds": round(t, 2)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


def per_gpu_rows(rows, steps: int):
    """Per-rank rates from shard.gather_floats rows [elapsed_s, payload bytes,
    serialize execute ms, deserialize execute ms, algorithmic bytes per
    launch]: each GPU's own payload GiB/s over its own timed span and its
    slower execute against the HBM roofline."""
    out = []
    for r, row in enumerate(rows):
        el, nbytes = row[0], row[1]
        o = {"rank": r, "GiBps": round(2.0 * nbytes * steps / el / GIB, 2), "payload_bytes": int(nbytes)}
        if len(row) == 5:
            ms, alg = max(row[2], row[3]), row[4]
            o["execute_GBps"] = round(alg / (ms * 1e-3) / 1e9, 1)
            o["frac"] = round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        out.append(o)
    return out


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: this process
    makes no HIP call (torch is never imported here) and starts N fresh
    worker processes of this same script, one per GPU, with the environment
    torchrun would give them (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on
    127.0.0.1). Rank 0 prints the one JSON line; the exit status is the
    first failing rank's. If a rank fails, the others (blocked in a
    bookkeeping barrier) are given 30 s and then killed by PID."""
    import signal
    import subprocess
    port = _free_port()
    procs = []

    def stop(signum, frame):
        # a launcher that signals this process (a time limit) ends the ranks too
        for p in procs:
            if p.poll() is None:
                p.kill()
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CFWS_BENCH_LAUNCHER="spawn")
        env.setdefault("GLOO_SOCKET_IFNAME", "lo")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=None if r == 0 else sys.stderr.fileno()))
    rc, failed_at = 0, None
    while any(p.poll() is None for p in procs):
        for p in procs:
            if p.returncode not in (None, 0) and rc == 0:
                rc, failed_at = p.returncode, time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > 30:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    for p in procs:
        if p.returncode != 0 and rc == 0:
            rc = p.returncode
    return 0 if rc == 0 else (rc if rc > 0 else 1)


def init_ranks(args):
    """(rank, world, device) of this process. One process per GPU: under
    torchrun, under spawn_ranks, or alone (N = 1). The bookkeeping
    collectives (the timing barriers, a max and a gather of a few CPU
    scalars) run over gloo on every box: the data path has no collective
    (SURVEY.md §8e), so RCCL is never initialised. CFWS_BENCH_REHEARSE=1:
    more ranks than GPUs (ranks share devices) -- a check of the multi-rank
    path on a smaller box, not a measurement."""
    import torch
    import torch.distributed as dist

    from coldforce_amd import cfws, shard
    rank, local_rank, world = shard.world()
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: running {world} ranks",
              file=sys.stderr)
    if args.dry_run:
        dev = None
    else:
        ngpu = torch.cuda.device_count()
        rehearse = os.environ.get("CFWS_BENCH_REHEARSE") == "1"
        if local_rank >= ngpu and not rehearse:
            sys.exit(f"bench.py: rank {rank} has no GPU ({ngpu} visible)")
        gpu = local_rank % ngpu
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        # gloo announces its connections on fd 1: keep stdout for the one
        # JSON line by sending fd 1 to stderr while the group forms
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    if dev is not None:
        cfws.init()
    return rank, world, dev


def launcher_name(world: int) -> str:
    """How this rank was started: "spawn" (spawn_ranks), "torchrun", or
    "single" (one process, N = 1)."""
    return os.environ.get("CFWS_BENCH_LAUNCHER", "torchrun" if "WORLD_SIZE" in os.environ else "single")


def bench_dry(args, rank, world):
    """--dry-run: the launch and bookkeeping of a multi-rank run with no GPU
    (the CPU test of spawn_ranks / torchrun): each rank builds its shard's
    descriptors on the host, times that, and the ranks meet in the same
    barrier / max / gather the GPU workloads use. The line carries no rate
    of the metric ("value": null)."""
    from coldforce_amd import shard
    t0 = time.perf_counter()
    for _ in range(args.warmup + args.steps):
        desc, _ = shard.uniform_shard(args.frames, args.frame_size, KEY_SEED, rank, world)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local)
    rows = shard.gather_floats([local, len(desc) * args.frame_size])
    line = {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "dry_run": True, "launcher": launcher_name(world),
            "config": {"workload": f"dry run: {args.frames} x {size_label(args.frame_size)} descriptors per rank"},
            "per_gpu": per_gpu_rows(rows, args.steps), "verified": True}
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import numpy as np
    import torch
    import torch.distributed as dist

    from coldforce_amd import cfws, shard
    from coldforce_amd import workloads as W

    rank, world, dev = init_ranks(args)
    if args.dry_run:
        rc = bench_dry(args, rank, world)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(rc)

    F, fs = args.frames, args.frame_size
    if args.workload in ("config5", "split", "accept", "index"):
        fn = {"config5": bench_h2, "split": bench_split, "accept": bench_accept,
              "index": bench_index}[args.workload]
        rc = fn(args, rank, world, dev)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(rc)
    flags = 0
    if args.workload == "config3":
        # each rank: its byte-balanced share (cut on message boundaries) of
        # one global Zipf batch of 4 GiB x world; world 1 is
        # config 3 itself
        c3 = W.CONFIG3
        desc_np, msgs, byte_base = shard.zipf_shard(c3["target_bytes"], rank, world, c3["seed"],
                                                    c3["key_seed"])
        arena_bytes = int(msgs["arena_bytes"])
        payload = torch.empty(W.round16(arena_bytes), dtype=torch.uint8, device=dev)
        cfws.fill_splitmix(payload, c3["seed"], byte_base)
        flags = cfws.DESERIALIZE_REASSEMBLE
        F = len(desc_np)
    elif args.workload == "config4":
        # one 8-way shard of the 8 M-frame batch per GPU (64 GiB payload +
        # 64 GiB wire + 64 GiB unmasked copy resident in HBM)
        c4 = CONFIG4
        if world > c4["shards"]:
            sys.exit("bench.py: config4 has 8 shards")
        F = c4["frames_total"] // c4["shards"]
        desc_np, byte_base = shard.uniform_shard(F, fs, c4["key_seed"], rank, c4["shards"])
        arena_bytes = F * fs
        payload = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
        cfws.fill_splitmix(payload, c4["payload_seed"], byte_base)
    else:
        desc_np, byte_base = shard.uniform_shard(F, fs, KEY_SEED, rank, world)
        arena_bytes = F * fs
        payload = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
        cfws.fill_splitmix(payload, PAYLOAD_SEED, byte_base)
    offs, wire_total = W.wire_layout(desc_np)
    wire = torch.empty(W.round16(wire_total), dtype=torch.uint8, device=dev)
    # config2 frames of a size that is not a multiple of 16: the packed
    # receive (align 16) places payload i at i * round16(fs)
    pstride = W.round16(fs) if args.workload == "config2" else fs
    back = torch.empty(payload.numel() + F * (pstride - fs) + 64, dtype=torch.uint8, device=dev)
    desc_ser = cfws.desc_to_device(desc_np, dev)
    desc_de = torch.empty((F, 32), dtype=torch.uint8, device=dev)
    status = torch.empty(F, dtype=torch.int32, device=dev)
    index = torch.from_numpy(offs.astype("int64")).to(dev)
    ws_ser = cfws.workspace(F, wire.numel(), dev)
    ws_de = cfws.workspace(F, back.numel(), dev)
    tot_ser = torch.zeros(1, dtype=torch.int64, device=dev)
    tot_de = torch.zeros(1, dtype=torch.int64, device=dev)

    # Each direction is one batch call (cfws_serialize_batch,
    # cfws_deserialize_batch), and the timed kernel is the call's streaming
    # pass, bracketed by events the library records right around its launch
    # (cfws_time_next_pass): the execute kernel after the plan, or for
    # batches of small frames (<= 512 B of wire per frame, no reassembly) the
    # fused plan + copy kernel of the receive,
    # deserialize_plan_single_kernel<true>
    if args.recv_uniform:
        if args.recv_scatter or args.workload != "config2":
            sys.exit("bench.py: --recv-uniform is a config2 slot receive (no --recv-scatter)")
        args.recv_slots = args.recv_info = True
    slot = W.round16(max(fs, 16)) if args.recv_slots or args.recv_scatter else 0
    if slot and (flags or slot != fs):
        sys.exit("bench.py: --recv-slots / --recv-scatter need config2 with a frame size that is a multiple of 16")
    # --recv-scatter: frame i to slot perm[i] (a seeded shuffle)
    perm = (torch.from_numpy(np.random.default_rng(5).permutation(F).astype(np.int64)).to(dev)
            if args.recv_scatter else None)
    dst_off = perm * slot if perm is not None else None
    if args.recv_info and not slot:
        sys.exit("bench.py: --recv-info needs --recv-slots or --recv-scatter")
    uniform = args.send == "uniform"
    if uniform and args.workload != "config2":
        sys.exit("bench.py: --send uniform needs config2 (a uniform batch)")
    keys_t = torch.from_numpy(desc_np["mask_key"].view(np.int32).copy()).to(dev) if uniform else None
    info_t = torch.empty((F, 8), dtype=torch.uint8, device=dev) if args.recv_info else None
    stride = wire_total // F if args.recv_uniform else 0       # a uniform batch: W per frame
    mismatch_t = torch.zeros(1, dtype=torch.int32, device=dev) if args.recv_uniform else None
    # the receive kernel the timed pass is, as the library routes the call
    recv_kernel = cfws.lib().cfws_deserialize_pass_kernel(F, wire_total, 16, flags, back.numel()).decode()

    def step(ev=None):
        if ev: cfws.time_next_pass(ev[0], ev[1])
        if uniform:
            cfws.serialize_uniform(payload, keys_t, F, fs, wire, opcode=cfws.OPCODE_BINARY, mask=True,
                                   total_t=tot_ser)
        else:
            cfws.serialize(payload, desc_ser, wire, ws_ser, tot_ser)
        if flags:
            # reassembly: two streaming passes (data frames, then control
            # frames), timed together after the plan
            cfws.deserialize_plan(wire, wire_total, index, desc_de, status, back.numel(), tot_de,
                                  ws_de, align=16, flags=flags)
            if ev: ev[2].record()
            cfws.deserialize_execute(wire, desc_de, status, back, ws_de, flags=flags)
            if ev: ev[3].record()
        else:
            if ev: cfws.time_next_pass(ev[2], ev[3])
            if dst_off is not None and info_t is not None:
                cfws.deserialize_scatter_info(wire, wire_total, index, dst_off, back, slot, info_t)
            elif dst_off is not None:
                cfws.deserialize_scatter(wire, wire_total, index, dst_off, back, slot, desc_de, status)
            elif stride:
                cfws.deserialize_slots_uniform(wire, wire_total, F, stride, back, slot, info_t, tot_de,
                                               mismatch_t)
            elif slot and info_t is not None:
                cfws.deserialize_slots_info(wire, wire_total, index, back, slot, info_t, tot_de)
            elif slot:
                cfws.deserialize_slots(wire, wire_total, index, back, slot, desc_de, status, tot_de)
            else:
                cfws.deserialize(wire, wire_total, index, back, desc_de, status, ws_de, tot_de, align=16)

    for _ in range(args.warmup):
        step()
    events = [[cfws.TimingEvent() for _ in range(4)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    local = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(local, dev)

    # correctness of what was timed: unmask(mask(P)) == P, every frame COMPLETE
    if info_t is not None:
        # the compact entries: payload_size, fin 1, opcode BINARY, status COMPLETE
        exp = fs | 1 << 32 | cfws.OPCODE_BINARY << 40
        ok_info = bool((info_t.view(torch.int64).view(-1) == exp).all().item())
        if mismatch_t is not None:
            ok_info = ok_info and int(mismatch_t.item()) == 0
        status.fill_(0 if ok_info else 1)
        if perm is None:
            tot_de.fill_(arena_bytes)
    if perm is not None:
        # frame i's payload is slot perm[i]: gather the slots back into frame order
        got = back[:arena_bytes].view(F, slot)[perm]
        verified = (int(tot_ser.item()) == wire_total and bool((status == 0).all().item())
                    and torch.equal(got.reshape(-1), payload[:arena_bytes]))
        del got
    elif pstride != fs and not slot:
        verified = (int(tot_ser.item()) == wire_total and int(tot_de.item()) == F * pstride
                    and bool((status == 0).all().item())
                    and torch.equal(back[:F * pstride].view(F, pstride)[:, :fs], payload[:arena_bytes].view(F, fs)))
    else:
        verified = (int(tot_ser.item()) == wire_total and int(tot_de.item()) == arena_bytes
                    and bool((status == 0).all().item())
                    and torch.equal(back[:arena_bytes], payload[:arena_bytes]))
    verified = shard.sum_over_ranks(1.0 if verified else 0.0, dev) == world

    # practical ceiling: a bare streaming copy of the same byte count
    # (cfws_device_copy: the best shape of tools/copy_probe.hip), and
    # torch's copy_ beside it
    def copy_rate(fn, reps=5):
        fn()
        c0, c1 = cfws.TimingEvent(), cfws.TimingEvent()
        c0.record()
        for _ in range(reps):
            fn()
        c1.record()
        torch.cuda.synchronize()
        ms = c0.elapsed_time(c1) / reps
        del c0, c1
        return 2 * payload.numel() / (ms * 1e-3) / 1e9

    n_copy = payload.numel() // 16 * 16
    copy_gbps = copy_rate(lambda: cfws.device_copy(payload, back, n_copy))
    torch_copy_gbps = copy_rate(lambda: back[:payload.numel()].copy_(payload))

    ser_each = [e[0].elapsed_time(e[1]) for e in events]
    de_each = [e[2].elapsed_time(e[3]) for e in events]
    ser_ms, de_ms = sum(ser_each) / args.steps, sum(de_each) / args.steps
    del events                               # HIP events freed while the runtime is up
    hdr = int(wire_total - arena_bytes)
    alg_bytes = 2 * arena_bytes + hdr       # read n + write n (+ headers) per launch
    # ms: the mean over the timed steps (what rocprof's average compares
    # with; roofline.achieved uses it), median_ms: SURVEY.md §8(d)'s median
    kern = {
        "serialize_execute": {"ms": round(ser_ms, 4), "median_ms": round(statistics.median(ser_each), 4),
                              "GBps": round(alg_bytes / (ser_ms * 1e-3) / 1e9, 1)},
        "deserialize_execute": {"ms": round(de_ms, 4), "median_ms": round(statistics.median(de_each), 4),
                                "GBps": round(alg_bytes / (de_ms * 1e-3) / 1e9, 1)},
    }
    dom_name = "serialize_execute" if ser_ms >= de_ms else "deserialize_execute"
    dom_ms = max(ser_ms, de_ms)
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    kernel_symbol = ((cfws.lib().cfws_serialize_uniform_pass_kernel(fs, 1).decode() if uniform
                      else "xform_kernel<0>")
                     if dom_name == "serialize_execute"
                     else cfws.lib().cfws_deserialize_slots_pass_kernel(F, wire_total, slot).decode() if slot
                     else recv_kernel if not flags else "xform_kernel<1>")
    # the PMC summary a traffic figure may come from: the same workload only
    traffic_key = (f"config2:{F}x{fs}" + (":uniform" if uniform else "")
                   + (":scatter" if perm is not None else ":slots" if slot else "")
                   + (":info" if info_t is not None else "") + (":implicit" if stride else "")
                   if args.workload == "config2" else
                   "config3" if args.workload == "config3" else f"config4:{F}x{fs}")
    rows = shard.gather_floats([local, arena_bytes, ser_ms, de_ms, alg_bytes], dev)
    total_payload = 2.0 * sum(r[1] for r in rows) * args.steps
    line = {
        "metric": METRIC,
        "value": round(total_payload / elapsed / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 payloads, glibc random() mask keys as co_ws_frame_serialize draws them)",
        "config": {
            "workload": (f"config2: {F} binary frames x {size_label(fs)} per GPU, client-mask "
                         f"(serialize) then server-unmask (deserialize), device resident"
                         + ("; the send through cfws_serialize_uniform (payload + one key per frame, "
                            "no plan)" if uniform else "")
                         + (f"; the receive to a shuffled order of {slot} B slots (cfws_deserialize_scatter"
                            f"{'_info' if info_t is not None else ''})"
                            if perm is not None else
                            f"; the receive into fixed {slot} B payload slots (cfws_deserialize_slots"
                            f"{'_uniform: no index' if stride else '_info' if info_t is not None else ''})"
                            if slot else "")
                         if args.workload == "config2" else
                         f"config4: shard {rank} of 8 of the 8 M x 64 KiB batch ({F} frames, "
                         f"64 GiB per GPU), client-mask then server-unmask, device resident"
                         if args.workload == "config4" else
                         f"config3: {F} frames / {len(msgs['len'])} Zipf messages (64 B-1 MiB, "
                         f"1-8 fragments) on rank 0, its byte-balanced share of a 4 GiB x "
                         f"{world} batch, client-mask then server-unmask with continuation "
                         f"reassembly, device resident"),
            "frames_per_gpu": F,
            "payload_bytes_per_gpu": arena_bytes,
            "wire_bytes_per_gpu": wire_total,
            "parallelism": f"shard-per-gpu x{world} (no collective)",
            "launcher": launcher_name(world),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kernel_symbol,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": load_traffic(kernel_symbol, traffic_key),
            "algorithmic_bytes_per_launch": alg_bytes,
            "avg_launch_ms": round(dom_ms, 4),
        },
        "kernels": kern,
        "per_gpu": per_gpu_rows(rows, args.steps),
        "copy_ceiling": {"GBps": round(copy_gbps, 1), "frac_of_copy": round(achieved / copy_gbps, 4),
                         "how": "cfws_device_copy of the payload arena, device to device (nt loads "
                                "and stores, 2 KiB per wave, 4 WG/CU: tools/copy_probe.hip's best "
                                "shape)",
                         "torch_copy_GBps": round(torch_copy_gbps, 1)},
        "verified": verified,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "config2":
        line["cpu_baseline"] = cpu_baseline(fs, args.cpu_seconds)
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not verified:
        sys.exit(1)


if __name__ == "__main__":
    main()
