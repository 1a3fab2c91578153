#!/bin/bash
# Bench-only A/B, alternating builds: in-tree library vs
# build/variants/libcfws_<VARIANT>.so, REPS rounds of one bench line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-bab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-3}); do
  for v in base ${VARIANT}; do
    if [ $v = base ]; then L=$PWD/coldforce_amd/libcfws.so; else L=$PWD/build/variants/libcfws_$v.so; fi
    CFWS_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --workload ${WL:-config2} ${ARGS} >> "$OUT/bench_$v.jsonl" 2>> "$OUT/err.txt" || exit 1
  done
done
echo "exit 0"
