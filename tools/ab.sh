#!/bin/bash
# A/B of build variants (build/variants/libcfws_<name>.so) on the bench workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
    CFWS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        > "$OUT/${v}_r$round.json" 2> "$OUT/${v}_r$round.err" || { echo "variant $v failed"; exit 1; }
  done
done
echo done
