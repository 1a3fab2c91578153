"""Summarise tools/ab.sh output: bench value and execute rates per variant."""
import glob, json, os, sys, collections
d = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f).rsplit("_r", 1)[0]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    k = j.get("kernels", {})
    rows[name].append((j["value"], k.get("serialize_execute", {}).get("GBps"),
                       k.get("deserialize_execute", {}).get("GBps"), j.get("verified")))
for name, rs in rows.items():
    print(f"{name:28s} " + "  |  ".join(f"{v:8.1f} GiB/s ser {s} deser {de} ok={ok}" for v, s, de, ok in rs))
