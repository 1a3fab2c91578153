#!/bin/bash
# Round 6's closing evidence on one box: tools/round_check.sh (GPU suite,
# smoke, default bench line with the CPU baseline, torchrun line, rocprof
# stats + PMC passes of config 2), then the config-3 and config-5 lines and
# the compact small-frame step (uniform send + receive without an index).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06fin}
OUT=gpurun_out/$T
mkdir -p "$OUT"
TAG=$T bash tools/round_check.sh > "$OUT/round_check.txt" 2>&1 &&
timeout -k 10 300 python3 bench.py --workload config3 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" &&
timeout -k 10 300 python3 bench.py --workload config5 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" &&
timeout -k 10 300 python3 bench.py --frames 16777216 --frame-size 256 --send uniform --recv-uniform \
    --no-cpu-baseline > "$OUT/fs256_implicit.json" 2> "$OUT/fs256_implicit.err"
rc=$?
echo "exit $rc"
exit $rc
