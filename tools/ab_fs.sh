#!/bin/bash
# Build variants (VARIANTS, build/variants/libcfws_<v>.so; base = in-tree)
# across uniform frame sizes (SIZES, 4 GiB of payload each), config-2 shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab_fs}
mkdir -p "$OUT"
for fs in ${SIZES:-16384 32768 65536 262144 1048576}; do
  fr=$((4294967296 / fs))
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
    CFWS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        --frames $fr --frame-size $fs > "$OUT/${v}_fs${fs}.json" 2> "$OUT/${v}_fs${fs}.err" || { echo "variant $v fs $fs failed"; exit 1; }
  done
done
echo done
