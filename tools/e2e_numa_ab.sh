#!/bin/bash
# NUMA placement A/B on one box: bench_e2e.py unbound (the OS's choice),
# bound to node 0 (the GPU's node on this pool) and to node 1, for config 2
# and config 5, twice. bench_e2e.py --numa-node binds before HIP loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-numaab}
mkdir -p "$OUT"
cat /sys/class/drm/card*/device/numa_node > "$OUT/gpu_numa.txt" 2>/dev/null
for r in 1 2; do
  for wl in config2 config5; do
    for n in -1 0 1; do
      timeout -k 10 300 python bench_e2e.py --workload $wl --numa-node $n > "$OUT/${wl}_n${n}_$r.json" 2>> "$OUT/err.txt" || exit 1
    done
  done
done
echo "exit 0"
