#!/bin/bash
# Streaming occupancy by frame size: CFWS_OCC_FRAME_MAX=0 (the per-mode
# reservations always) vs 65536 (register-limited residency for every batch
# averaging <= 64 KiB per frame), two rounds, across frame sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-occ}; mkdir -p "$OUT"
run() {
  local name=$1; shift
  for round in 1 2; do
    for o in 0 65536; do
      CFWS_OCC_FRAME_MAX=$o timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" \
        > "$OUT/${name}_m${o}_r$round.json" 2> "$OUT/${name}_m${o}_r$round.err" || { echo "$name $o failed"; exit 1; }
    done
  done
}
case "${SET:-1}" in
1)
  run fs1k --frames 4194304 --frame-size 1024
  run fs4k --frames 1048576 --frame-size 4096
  run fs8k --frames 524288 --frame-size 8192
  run fs16k --frames 262144 --frame-size 16384
  run config3 --workload config3
  run config5 --workload config5 ;;
2)
  run fs2k --frames 2097152 --frame-size 2048
  run fs512 --frames 8388608 --frame-size 512 ;;
esac
echo done
