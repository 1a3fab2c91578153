#!/bin/bash
# Fused serialize (serialize_fused_kernel, the one-call default for <= 4 KiB of
# wire capacity per frame) against plan + execute (CFWS_FUSED_SER=0) on one
# box, alternating, two rounds, at 256 B / 1 KiB / 2 KiB / 3 KiB frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-fsab}
mkdir -p "$OUT"
for r in 1 2; do
  for fs in 256 1024 2048 3072; do
    F=$(( (4 << 30) / fs ))
    for fz in 1 0; do
      CFWS_FUSED_SER=$fz timeout -k 10 200 python bench.py --frames $F --frame-size $fs --no-cpu-baseline \
        > "$OUT/fs${fs}_fused${fz}_r$r.json" 2> "$OUT/fs${fs}_fused${fz}_r$r.err" || exit 1
    done
  done
done
echo done
