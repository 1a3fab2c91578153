#!/bin/bash
# Per-frame latency of the drop-in co_ws_frame_* API (oracle/_ref/dropin_link
# bench: serialize(mask) + deserialize of one frame, C, linked to libcfws.so)
# by frame size and path:
#   host     the size policy's calling-thread XOR (CFWS_DROPIN_GPU_MIN huge)
#   service  the frame service (frames <= 32 KiB by default; device forced)
#   launch   launch + synchronise per frame (CFWS_DROPIN_SERVICE=0: zero-copy
#            up to 1 MiB)
#   dma      H2D + kernel + D2H (CFWS_DROPIN_ZC_MAX=0)
# Each line has wall and CPU time per frame (the calling thread's, and the
# process's per serialize + deserialize pair).
# The size policy's default (CFWS_DROPIN_GPU_MIN_DEFAULT) follows from these:
# `host` wins on wall and on CPU time at every size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dropin}
mkdir -p "$OUT"
for mode in ${MODES:-host service launch dma}; do
  for size in ${SIZES:-125 1024 4096 16384 32768 65536 262144 1048576 4194304}; do
    n=4000; [ $size -ge 262144 ] && n=300; [ $size -ge 4194304 ] && n=60
    case $mode in
      host) env="CFWS_DROPIN_GPU_MIN=1000000000" ;;
      service) env="CFWS_DROPIN_GPU_MIN=0 CFWS_DROPIN_SERVICE_MAX=65536" ;;
      launch) env="CFWS_DROPIN_GPU_MIN=0 CFWS_DROPIN_SERVICE=0" ;;
      dma) env="CFWS_DROPIN_GPU_MIN=0 CFWS_DROPIN_SERVICE=0 CFWS_DROPIN_ZC_MAX=0" ;;
    esac
    [ $mode = service ] && [ $size -gt 65536 ] && continue
    line=$(env $env timeout -k 10 120 oracle/_ref/dropin_link bench $size $n) || exit 1
    echo "{\"path\": \"$mode\", ${line#\{}" >> "$OUT/dropin_lat.jsonl"
  done
done
echo done
