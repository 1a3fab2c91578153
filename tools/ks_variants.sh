#!/bin/bash
# rocprofv3 kernel stats of `bench.py $ARGS` (default --workload split) for the
# in-tree build and each build/variants/libcfws_$v.so in $VARIANTS.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-ks}; mkdir -p "$OUT"
for v in base $VARIANTS; do
  L=$R/coldforce_amd/libcfws.so; [ $v = base ] || L=$R/build/variants/libcfws_$v.so
  CFWS_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks_$v" -o ks -- \
    python3 $R/bench.py ${ARGS:---workload split} --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/ks_$v.log" 2>&1 || exit 1
done
