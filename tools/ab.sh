#!/bin/bash
# A/B of build variants (build/variants/libcfws_<name>.so; "base" = the
# in-tree library) x streaming-kernel LDS reservations (CFWS_XFORM_LDS, which
# sets workgroups per CU), two rounds, on the bench workload (WL, default
# config2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
    for lds in ${LDS:-default}; do
      if [ "$lds" = default ]; then unset CFWS_XFORM_LDS; else export CFWS_XFORM_LDS=$lds; fi
      CFWS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
          --no-cpu-baseline --workload ${WL:-config2} $ARGS \
          > "$OUT/${v}_lds${lds}_r$round.json" 2> "$OUT/${v}_lds${lds}_r$round.err" || { echo "variant $v lds $lds failed"; exit 1; }
    done
  done
done
echo done
