#!/bin/bash
# Send-side variants (build/variants/libcfws_$v.so) against the in-tree
# build over config 2, config 5, config 3 and 1 KiB frames, two alternating
# rounds; prints value and execute times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-send_ab}; mkdir -p "$OUT"
run() {
  local name=$1; shift
  for round in 1 2; do
    for v in base $VARIANTS; do
      L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
      CFWS_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" \
        > "$OUT/${name}_${v}_r$round.json" 2> "$OUT/${name}_${v}_r$round.err" || { echo "$name $v failed"; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/${name}_${v}_r$round.json').read().splitlines()[-1])
k=d.get('kernels') or {}; print('$name', '$v', 'r$round', d['value'], {a: b['ms'] for a, b in k.items()})"
    done
  done
}
run c2
run c5 --workload config5
run c3 --workload config3
run fs1k --frames 4194304 --frame-size 1024
