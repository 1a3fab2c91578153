"""Per-kernel means of every counter in the rocprofv3 --pmc passes under a
directory (counter_collection.csv files), plus derived per-wave figures.

usage: python3 tools/pmc_kernels.py <dir> [name-substring ...]
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    root = sys.argv[1]
    keep = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if keep and not any(s in k for s in keep):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.1f}")
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
                      "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    print(f"  per wave {c:22s} {m[c] / w:12.1f}")


if __name__ == "__main__":
    main()
