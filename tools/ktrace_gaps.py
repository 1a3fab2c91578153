"""Per-step kernel timeline (durations and the gaps between kernels) from a
rocprofv3 --kernel-trace CSV: the last `steps` steps, a step starting at
`first` (a kernel-name substring)."""
import csv
import sys


def main(path, first="serialize_plan_reduce", steps=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]
              and "deserialize" not in r["Kernel_Name"]]
    if len(starts) < steps + 1:
        sys.exit("not enough steps")
    i0, i1 = starts[-steps - 1], starts[-1]
    prev = None
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:40]
        print(f"{name:40s} {(e - s) / 1000:9.2f} us  gap {gap:6.2f} us")
        prev = e
    t = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1000 / steps
    print(f"step {t:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
