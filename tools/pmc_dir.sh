#!/bin/bash
# Counters of the config-2 streaming kernels (serialize xform<0> against
# deserialize xform<1>): instruction mix, L2 hit/miss and EA requests,
# L1 -> L2 requests and translation misses. One --pmc pass per block group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-pmcdir}
mkdir -p "$OUT"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o $1 -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$1.log" 2>&1
}
run sq "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" &&
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" &&
run tcp "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
echo "exit $?"
