#!/bin/bash
# GPU parity suite on one A/B build ($TESTLIB: build/variants/libcfws_<v>.so),
# then bench lines of the in-tree build and each variant in $VARIANTS on
# small frames, config 2 and config 3, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-vab}
mkdir -p "$OUT"
if [ -n "$TESTLIB" ]; then
  CFWS_LIB=$PWD/build/variants/libcfws_$TESTLIB.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
      --timeout 300 --timeout-method thread > "$OUT/pytest_$TESTLIB.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_$TESTLIB.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
for r in 1 2; do
  for v in base ${VARIANTS}; do
    L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
    for w in "fs1k --frames 4194304 --frame-size 1024" "fs256 --frames 16777216 --frame-size 256" "c2" "c3 --workload config3"; do
      set -- $w; name=$1; shift
      CFWS_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > "$OUT/${name}_${v}_r$r.json" 2> "$OUT/${name}_${v}_r$r.err" || { echo "$name $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${name}_${v}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('${name}_${v}_r$r', d['value'], k['serialize_execute']['ms'], k['deserialize_execute']['ms'])"
    done
  done
done
