#!/bin/bash
# Build-variant A/B on small frames (base = in-tree library vs
# build/variants/libcfws_$v.so for v in $VARIANTS), two alternating rounds:
# 4 M x 1 KiB, 16 M x 256 B, 1 M x 4 KiB (4 GiB of payload each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-small_ab}; mkdir -p "$OUT"
for w in ${WL:-fs1k:4194304:1024 fs256:16777216:256 fs4k:1048576:4096}; do
  set -- ${w//:/ }
  for round in $(seq ${ROUNDS:-2}); do
    for v in base $VARIANTS; do
      L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
      A="--frames $2 --frame-size $3"; [ "$2" = w ] && A="--workload $3"     # name:w:config3
      CFWS_LIB=$L timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $A \
        > "$OUT/${1}_${v}_r$round.json" 2> "$OUT/${1}_${v}_r$round.err" || { echo "$1 $v failed"; exit 1; }
      echo "$1 $v r$round $(python3 -c "import json;d=json.loads(open('$OUT/${1}_${v}_r$round.json').read().splitlines()[-1]);print(d['value'], d['kernels']['serialize_execute']['ms'], d['kernels']['deserialize_execute']['ms'])")"
    done
  done
done
