#!/bin/bash
# rocprofv3 kernel stats of configs 3 and 5 (and 1 KiB frames) on the current build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-config_kstats}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o k -- python3 $R/bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o k -- python3 $R/bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fs1k -o k -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/fs1k.json 2> $OUT/fs1k.err
