#!/bin/bash
# Small-batch latency and kernel stats of the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-small_now}; mkdir -p $OUT
timeout -k 10 300 python tools/graph_latency.py --sizes 1,16,256,1024 > $OUT/lat.jsonl 2> $OUT/lat.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o k -- python3 $GRAFT_REPO_ROOT/tools/graph_latency.py --sizes 256 --iters 100 > $GRAFT_REPO_ROOT/$OUT/prof.txt 2>&1
