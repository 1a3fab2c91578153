#!/bin/bash
# HBM traffic of config 5's two streaming kernels (send xform<3>, receive
# xform<1>): FETCH_SIZE and WRITE_SIZE in separate --pmc passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-pmc5}
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o $c -- \
    python3 $R/bench.py --no-cpu-baseline --workload config5 --steps 2 --warmup 1 > "$OUT/$c.log" 2>&1 || exit 1
done
echo "exit 0"
