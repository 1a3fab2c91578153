#!/bin/bash
# Serialize in-region edge chunks A/B (CFWS_SER_INREG=1 vs 0, with
# profiles/r03_inreg_ab/inreg_edges.patch applied; the knob is gone from the
# tree): GPU parity suite first, then bench lines per workload, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-inreg}
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
run() {  # name knob args...
  local name=$1 k=$2; shift 2
  CFWS_SER_INREG=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -3 "$OUT/$name.err"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['kernels'])"
}
for r in 1 2; do
  for k in 1 0; do
    run fs1k_k${k}_r$r $k --frames 4194304 --frame-size 1024
    run fs256_k${k}_r$r $k --frames 16777216 --frame-size 256
    run fs2k_k${k}_r$r $k --frames 2097152 --frame-size 2000
    run c2_k${k}_r$r $k
    run c3_k${k}_r$r $k --workload config3
  done
done
echo done
