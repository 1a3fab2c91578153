#!/bin/bash
# Counters for config 5's receive-plan kernels (h2_msg_parse against
# h2_de_plan_reduce / h2_units, which do similar dependent loads in a fifth of
# the time): waves, VMEM instructions and wave cycles, L2 hits / misses, and
# vector-L1 address translation hits / misses. One --pmc pass per group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-pmcparse}
mkdir -p "$OUT"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o $1 -- \
    python3 $R/bench.py --no-cpu-baseline --workload config5 --steps 2 --warmup 1 > "$OUT/$1.log" 2>&1
}
run sq "SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" &&
run utcl "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
echo "exit $?"
