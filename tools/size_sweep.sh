#!/bin/bash
# The final build across uniform frame sizes (4 GiB of payload each, mask
# then unmask, device resident) plus configs 3 and 5: one bench line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-size_sweep}; mkdir -p "$OUT"
for fs in 256 512 1024 2048 4096 16384 65536 262144 1048576; do
  timeout -k 10 300 python bench.py --frames $((4294967296 / fs)) --frame-size $fs --steps 20 --warmup 10 \
      --no-cpu-baseline > "$OUT/fs$fs.json" 2> "$OUT/fs$fs.err" || { echo "fs $fs failed"; exit 1; }
done
timeout -k 10 300 python bench.py --workload config3 --no-cpu-baseline > "$OUT/config3.json" 2> "$OUT/config3.err" &&
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > "$OUT/config5.json" 2> "$OUT/config5.err" &&
timeout -k 10 300 python bench.py --workload config5 --frame-size 65536 --no-cpu-baseline > "$OUT/config5_64k.json" 2> "$OUT/config5_64k.err"
