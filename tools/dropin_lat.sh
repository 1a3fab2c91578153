#!/bin/bash
# Per-frame latency of the drop-in co_ws_frame_* API (oracle/_ref/dropin_link
# bench: serialize(mask) + deserialize of one frame, C, linked to libcfws.so)
# by frame size: the frame service (default, frames <= 64 KiB), the launch +
# synchronise path (CFWS_DROPIN_SERVICE=0: zero-copy up to 1 MiB), and the
# DMA path (CFWS_DROPIN_SERVICE=0 CFWS_DROPIN_ZC_MAX=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dropin}
mkdir -p "$OUT"
for mode in service launch dma; do
  for size in 125 1024 16384 65536 262144 1048576; do
    n=4000; [ $size -ge 262144 ] && n=300
    case $mode in
      service) env= ;;
      launch) env="CFWS_DROPIN_SERVICE=0" ;;
      dma) env="CFWS_DROPIN_SERVICE=0 CFWS_DROPIN_ZC_MAX=0" ;;
    esac
    line=$(env $env timeout -k 10 120 oracle/_ref/dropin_link bench $size $n) || exit 1
    echo "{\"path\": \"$mode\", ${line#\{}" >> "$OUT/dropin_lat.jsonl"
  done
done
echo done
