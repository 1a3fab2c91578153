#!/bin/bash
# ws_accept_kernel occupancy: the default (4 waves/SIMD by registers) against
# __launch_bounds__ minimum blocks 6 and 8 (80 / 64 VGPRs, with spills).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_acc2; mkdir -p $OUT
for r in 1 2; do
  for v in base acc6 acc8; do
    if [ $v = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
    CFWS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload accept --no-cpu-baseline > $OUT/${v}_$r.json 2>/dev/null || exit 1
  done
done
