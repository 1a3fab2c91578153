#!/bin/bash
# rocprofv3 --pmc passes (one run each) over `bench.py $ARGS`: PASSES holds
# the counter sets separated by ';'. Summary: python3 tools/pmc_kernels.py
# gpurun_out/$TAG [kernel-substring ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-pmc}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra SETS <<< "$PASSES"
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o p -- \
    python3 $R/bench.py ${ARGS:---workload split} --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || exit 1
done
