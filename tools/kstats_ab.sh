#!/bin/bash
# rocprof kernel stats + bench line of one workload for the in-tree library
# and a variant (build/variants/libcfws_<VARIANT>.so), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-kab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base ${VARIANT:-presplit}; do
  if [ $v = base ]; then L=$R/coldforce_amd/libcfws.so; else L=$R/build/variants/libcfws_$v.so; fi
  CFWS_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --workload ${WL:-config5} > "$OUT/bench_$v.json" 2>/dev/null || exit 1
  ( cd /tmp && CFWS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o kt -- \
      python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload ${WL:-config5} ) > "$OUT/$v.log" 2>&1 || exit 1
done
echo done
