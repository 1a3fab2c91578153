#!/bin/bash
# Where the 1 KiB-frame streaming kernels spend their cycles: three --pmc
# passes (instruction mix, wait/active cycles, levels) over
# `bench.py --frames 4194304 --frame-size 1024`, edge chunks in a launch of
# their own (CFWS_EDGE_SPLIT=1) so the region kernels are counted alone.
# ARGS overrides the bench arguments (e.g. ARGS="--workload split").
# Summary: python3 tools/pmc_kernels.py gpurun_out/$TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-pmcfs1k}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
P3="SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_LEVEL_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_RD"
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  CFWS_EDGE_SPLIT=${EDGE_SPLIT:-1} timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o p -- \
    python3 $R/bench.py ${ARGS:---frames 4194304 --frame-size 1024} --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || exit 1
done
