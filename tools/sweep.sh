#!/bin/bash
# Grid-size sweep of the streaming kernel (CFWS_GRID = max workgroups).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p "$OUT"
for g in ${GRIDS:-2048 4096 8192 16384 65536 262144}; do
  CFWS_GRID=$g timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/grid_$g.json" 2> "$OUT/grid_$g.err" || { echo "grid $g failed"; exit 1; }
done
echo done
