#!/bin/bash
# Per-frame latency of the drop-in co_ws_frame_* API (oracle/_ref/dropin_link
# bench: serialize(mask) + deserialize of one frame, C, linked to libcfws.so),
# zero-copy path (default) vs the DMA path (CFWS_DROPIN_ZC_MAX=0), by size.
# (Polling hipStreamQuery instead of hipStreamSynchronize measured 2 us
# slower per frame.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dropin}
mkdir -p "$OUT"
for zc in default 0; do
  for size in 125 1024 16384 65536 262144 1048576 4194304; do
    n=2000; [ $size -ge 262144 ] && n=300
    if [ $zc = default ]; then
      timeout -k 10 120 oracle/_ref/dropin_link bench $size $n >> "$OUT/zc.jsonl" || exit 1
    else
      CFWS_DROPIN_ZC_MAX=0 timeout -k 10 120 oracle/_ref/dropin_link bench $size $n >> "$OUT/dma.jsonl" || exit 1
    fi
  done
done
echo done
