#!/bin/bash
# tools/phase_probe.py timed, then its FETCH_SIZE / WRITE_SIZE per dispatch
# (separate rocprofv3 passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-phase}; mkdir -p $OUT
cd $R && timeout -k 10 300 python tools/phase_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || exit 1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o p -- python3 $R/tools/phase_probe.py --reps 3 > $OUT/pmc_$c.log 2>&1 || exit 1
done
