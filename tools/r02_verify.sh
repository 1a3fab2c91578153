#!/bin/bash
# The default build after the round-2 kernel changes: GPU parity suite, then
# the bench on configs 2 (with the CPU baseline), 3 and 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r02_verify}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/c2.json 2> $OUT/c2.err &&
timeout -k 10 300 python bench.py --workload config3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err &&
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err
