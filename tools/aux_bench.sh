#!/bin/bash
# SURVEY.md 8(f) rows #2 and #4 measured: bench.py --workload accept / index
# (with their CPU baselines), rocprofv3 kernel stats of each, and the VALU
# instruction count of the accept-key kernel (one --pmc pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-aux}
mkdir -p $OUT
timeout -k 10 300 python bench.py --workload accept > $OUT/accept.json 2> $OUT/accept.err &&
timeout -k 10 300 python bench.py --workload index > $OUT/index.json 2> $OUT/index.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_accept -o kt -- python3 $R/bench.py --workload accept --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt_accept.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_index -o kt -- python3 $R/bench.py --workload index --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt_index.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d $OUT/pmc_accept -o pmc -- python3 $R/bench.py --workload accept --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_accept.log 2>&1
