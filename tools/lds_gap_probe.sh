#!/bin/bash
# Do the ~6 us gaps around the streaming launches come from the LDS
# reservation changing between consecutive kernels? Config 2 kernel traces
# with (a) defaults, (b) every kernel at 32,000 B (plans and both streams),
# (c) plans at 0 and streams at 32,000. SET=2: the streaming grid capped
# (CFWS_GRID, grid-stride over the regions). SET=3: every plan kernel and
# both streams at 96 VGPRs (a -DCFWS_VGPR_PAD_ON build, since removed: no
# change). SET=4: steps with no timing events (tools/noevent_steps.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-ldsgap}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o kt -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
case "${SET:-1}" in
1)
  run a CFWS_PLAN_LDS=0
  run b CFWS_PLAN_LDS=32000 CFWS_XFORM_LDS=32000
  run c CFWS_PLAN_LDS=0 CFWS_XFORM_LDS=32000 ;;
3)
  run base CFWS_PLAN_LDS=0 ;;
4)
  CFWS_PLAN_LDS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/noev -o kt -- python3 $R/tools/noevent_steps.py 12 > $OUT/noev.txt 2>&1 || exit 1 ;;
2)
  run g8k CFWS_GRID=8192
  run g32k CFWS_GRID=32768
  run g131k CFWS_GRID=131072 ;;
esac
