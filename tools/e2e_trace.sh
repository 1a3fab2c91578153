#!/bin/bash
# Timeline of the host-to-host pipeline (bench_e2e.py): kernel + memory-copy
# trace, no counters. Reduced reps; tools/e2e_timeline.py reads the CSVs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-e2etrace}
mkdir -p "$OUT"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT" -o tr -- python3 "$GRAFT_REPO_ROOT/bench_e2e.py" --workload ${WL:-config2} --reps 2 ) \
    > "$OUT/trace.txt" 2>&1
rc=$?
echo "exit $rc"
exit $rc
