#!/bin/bash
# Kernel stats of the 1 KiB-frame batch (4 M frames, config 1's frame size).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-fs1k}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k -- python3 $R/bench.py --frames ${FRAMES:-4194304} --frame-size ${FS:-1024} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
