#!/bin/bash
# Instruction mix of the 1 KiB-frame serialize with its edge chunks as a
# launch of their own (CFWS_EDGE_SPLIT=1): xform<0> (regions only) against
# edge_kernel<0>, one --pmc pass (4 M frames, 2 steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-pmcedges}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CFWS_EDGE_SPLIT=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM \
  --output-format csv -d "$OUT/sq" -o sq -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/sq.log" 2>&1
