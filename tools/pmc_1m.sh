#!/bin/bash
# HBM traffic of the streaming kernels at 1 MiB vs 64 KiB frames (4 GiB
# each): FETCH_SIZE and WRITE_SIZE, separate passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-pmc1m}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for fs in 65536 1048576; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/fs${fs}_$c -o p -- python3 $R/bench.py --frames $((4294967296 / fs)) --frame-size $fs --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fs${fs}_$c.log 2>&1 || exit 1
  done
done
