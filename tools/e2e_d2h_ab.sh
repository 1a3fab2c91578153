#!/bin/bash
# D2H leg A/B on one box: mapped host arenas with the kernel D2H (default),
# mapped with SDMA D2H (CFWS_PIPELINE_D2H=dma), torch pinned (SDMA), x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-d2hab}
mkdir -p "$OUT"
WL=${WL:-config2}
for r in 1 2; do
  timeout -k 10 300 python bench_e2e.py --workload $WL --host mapped > "$OUT/${WL}_mapped_kernel_$r.json" 2>> "$OUT/err.txt" &&
  CFWS_PIPELINE_D2H=dma timeout -k 10 300 python bench_e2e.py --workload $WL --host mapped > "$OUT/${WL}_mapped_dma_$r.json" 2>> "$OUT/err.txt" &&
  timeout -k 10 300 python bench_e2e.py --workload $WL --host torch > "$OUT/${WL}_torch_$r.json" 2>> "$OUT/err.txt" || exit 1
done
echo "exit 0"
