#!/bin/bash
# rocprofv3 kernel-trace + stats of bench.py for a workload (default config2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-kstats}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for w in ${WORKLOADS:-config2}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$w" -o kt -- \
      python3 $R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --workload $w > "$OUT/$w.log" 2>&1 || exit 1
done
echo done
