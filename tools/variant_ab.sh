#!/bin/bash
# Build-variant A/B (base = in-tree library vs build/variants/libcfws_$VARIANT.so)
# over a few workloads, two rounds: 1 KiB, 4 KiB, config 3, config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-variant_ab}; mkdir -p "$OUT"
run() {
  local name=$1; shift
  for round in 1 2; do
    for v in base $VARIANT; do
      L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
      CFWS_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" \
        > "$OUT/${name}_${v}_r$round.json" 2> "$OUT/${name}_${v}_r$round.err" || { echo "$name $v failed"; exit 1; }
    done
  done
}
run fs1k --frames 4194304 --frame-size 1024
run fs4k --frames 1048576 --frame-size 4096
run config3 --workload config3
run config2
echo done
