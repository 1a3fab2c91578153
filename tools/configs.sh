#!/bin/bash
# Device-resident benches of configs 3, 4 (one GPU's shard), 5 (16,376 B and
# 64 KiB frames), rocprof kernel stats of configs 3 and 5, and the
# host-to-host (PCIe-inclusive) rates of configs 2, 3, 5. One GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-configs}
mkdir -p "$OUT"
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B --workload config3 > "$OUT/config3_device.json" 2> "$OUT/config3.err" &&
timeout -k 10 600 $B --workload config4 --steps 10 > "$OUT/config4_shard_device.json" 2> "$OUT/config4.err" &&
timeout -k 10 300 $B --workload config5 > "$OUT/config5_device.json" 2> "$OUT/config5.err" &&
timeout -k 10 300 $B --workload config5 --frame-size 65536 > "$OUT/config5_64k_device.json" 2> "$OUT/config5_64k.err" &&
TAG=${TAG:-configs}/kstats WORKLOADS="config3 config5" bash tools/kstats.sh > "$OUT/kstats.txt" 2>&1 &&
timeout -k 10 300 python bench_e2e.py --workload config2 > "$OUT/e2e_config2.json" 2> "$OUT/e2e2.err" &&
timeout -k 10 300 python bench_e2e.py --workload config3 > "$OUT/e2e_config3.json" 2> "$OUT/e2e3.err" &&
timeout -k 10 300 python bench_e2e.py --workload config5 > "$OUT/e2e_config5.json" 2> "$OUT/e2e5.err"
rc=$?
echo "exit $rc"
exit $rc
