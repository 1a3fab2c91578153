#!/bin/bash
# Config 3 kernel stats with the edge chunks inside the streaming launch
# (default) and as launches of their own (CFWS_EDGE_SPLIT=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02_c3kt; mkdir -p $OUT
for sp in 0 1; do
  CFWS_EDGE_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/split$sp -o kt -- python3 $R/bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/split$sp.log 2>&1 || exit 1
done
