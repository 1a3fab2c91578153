"""Timeline of a host-pipeline run from rocprofv3 --kernel-trace
--memory-copy-trace CSVs (tools/e2e_trace.sh): every kernel and copy in
start order with its stream, duration and the gap since the previous event
of the same class (H2D copy / D2H copy / kernel), over a window.

  python tools/e2e_timeline.py <dir> [--from-kernel NAME --nth K --count N]
"""
import argparse
import csv
import glob
import os


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:40]


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            ev.append(dict(kind="K", name=short(r["Kernel_Name"]), stream=int(r["Stream_Id"]),
                           t0=int(r["Start_Timestamp"]), t1=int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            dirn = "H2D" if "HOST_TO_DEVICE" in r["Direction"] else (
                "D2H" if "DEVICE_TO_HOST" in r["Direction"] else r["Direction"][-14:])
            ev.append(dict(kind=dirn, name="copy " + dirn, stream=int(r["Stream_Id"]),
                           t0=int(r["Start_Timestamp"]), t1=int(r["End_Timestamp"])))
    ev.sort(key=lambda e: e["t0"])
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--from-kernel", default="copy_out_kernel")
    ap.add_argument("--nth", type=int, default=0, help="start at the K-th such kernel")
    ap.add_argument("--count", type=int, default=40)
    a = ap.parse_args()
    ev = load(a.dir)
    idx = [i for i, e in enumerate(ev) if e["name"].startswith(a.from_kernel)]
    if not idx:
        raise SystemExit("kernel not found")
    s = idx[min(a.nth, len(idx) - 1)]
    win = ev[s:s + a.count]
    base = win[0]["t0"]
    last_end = {}
    for e in win:
        cls = e["kind"]
        gap = (e["t0"] - last_end[cls]) / 1e3 if cls in last_end else 0.0
        last_end[cls] = max(last_end.get(cls, 0), e["t1"])
        print(f"{(e['t0'] - base) / 1e3:10.1f} us  {(e['t1'] - e['t0']) / 1e3:9.1f} us  "
              f"s{e['stream']:<3} {e['name']:<42} gap {gap:8.1f}")
    span = (win[-1]["t1"] - base) / 1e3
    busy = {}
    for e in win:
        busy[e["kind"]] = busy.get(e["kind"], 0) + (e["t1"] - e["t0"]) / 1e3
    print(f"window {span:.1f} us; busy " + ", ".join(f"{k} {v:.1f} us" for k, v in busy.items()))


if __name__ == "__main__":
    main()
