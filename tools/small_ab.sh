#!/bin/bash
# Small-batch latency A/B (tools/graph_latency.py) of the in-tree library vs
# build/variants/libcfws_<VARIANT>.so, plus rocprof kernel stats of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-smallab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base ${VARIANT:-cpt4}; do
  if [ $v = base ]; then L=$PWD/coldforce_amd/libcfws.so; else L=$PWD/build/variants/libcfws_$v.so; fi
  CFWS_LIB=$L timeout -k 10 300 python tools/graph_latency.py --sizes ${SIZES:-1,16,256,1024} > "$OUT/lat_$v.jsonl" 2>/dev/null || exit 1
  ( cd /tmp && CFWS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$v" -o k -- python3 "$GRAFT_REPO_ROOT/tools/graph_latency.py" --sizes 256 --iters 100 ) > "$OUT/prof_$v.txt" 2>&1 || exit 1
done
echo "exit 0"
