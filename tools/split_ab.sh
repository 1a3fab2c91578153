#!/bin/bash
# Split-op payload kernel variants (build/variants/libcfws_$v.so) against the
# in-tree build, `bench.py --workload split`, two alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-split_ab}; mkdir -p "$OUT"
for round in 1 2; do
  for v in base $VARIANTS; do
    L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
    CFWS_LIB=$L timeout -k 10 200 python bench.py --workload split --steps 20 --warmup 3 --no-cpu-baseline \
      > "$OUT/${v}_r$round.json" 2> "$OUT/${v}_r$round.err" || { echo "$v failed"; exit 1; }
    echo "$v r$round $(python3 -c "import json;print(json.loads(open('$OUT/${v}_r$round.json').read().splitlines()[-1])['value'])")"
  done
done
