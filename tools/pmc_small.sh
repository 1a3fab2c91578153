#!/bin/bash
# Instruction mix and LDS counters of the single-launch small-batch kernels
# (256 x 1 KiB frames, tools/graph_latency.py), one --pmc pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-pmcsmall}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  --output-format csv -d "$OUT/sq" -o sq -- python3 $R/tools/graph_latency.py --sizes 256 --iters 20 > "$OUT/sq.log" 2>&1
echo "exit $?"
