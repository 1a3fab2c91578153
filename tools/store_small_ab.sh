#!/bin/bash
# Serialize store-policy variants (build/variants/libcfws_<v>.so from
# `make variant V=<v> F=-DCFWS_STORE_AUX_SER=<bits>`) on small frames and
# config 2, two rounds; one bench line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-store_small}
mkdir -p "$OUT"
for r in 1 2; do
  for v in base ${VARIANTS}; do
    L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
    for w in "fs1k --frames 4194304 --frame-size 1024" "fs256 --frames 16777216 --frame-size 256" "c2"; do
      set -- $w; name=$1; shift
      CFWS_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > "$OUT/${name}_${v}_r$r.json" 2> "$OUT/${name}_${v}_r$r.err" || { echo "$name $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${name}_${v}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('${name}_${v}_r$r', d['value'], k['serialize_execute']['ms'], k['deserialize_execute']['ms'])"
    done
  done
done
