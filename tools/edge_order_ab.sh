#!/bin/bash
# Edge-workgroup order A/B (CFWS_EDGE_ORDER 0 = first, 1 = spread through the
# grid), two rounds, over workloads with few and many edge workgroups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-edge_order}; mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  for round in 1 2; do
    for o in 0 1; do
      CFWS_EDGE_ORDER=$o timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" \
        > "$OUT/${name}_o${o}_r$round.json" 2> "$OUT/${name}_o${o}_r$round.err" || { echo "$name o$o failed"; exit 1; }
    done
  done
}
case "${SET:-1}" in
1)
  run fs16k --frames 262144 --frame-size 16384
  run fs32k --frames 131072 --frame-size 32768
  run fs4k --frames 1048576 --frame-size 4096
  run config4 --workload config4 --steps 5 ;;
2)
  run fs1k --frames 4194304 --frame-size 1024
  run fs8k --frames 524288 --frame-size 8192
  run config3 --workload config3 ;;
esac
echo done
