#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel trace + stats, then HBM
# counters in separate passes (FETCH_SIZE and WRITE_SIZE do not fit one pass).
# ARGS: extra bench.py arguments (e.g. "--frames 4194304 --frame-size 1024").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH="$R/bench.py $ARGS --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 $BENCH > "$OUT/kt.log" 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/write.log" 2>&1
rc=$?
echo "exit $rc"
find "$OUT" -name '*.csv' | head -20
exit $rc
