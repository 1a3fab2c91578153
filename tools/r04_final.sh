#!/bin/bash
# Round-4 evidence from the final tree: GPU suite, smoke, the default bench
# line (and through torch.distributed.run), rocprof kernel stats and PMC
# HBM traffic for the headline, the other workloads' bench lines, config 1
# and the drop-in latency. Every GPU step has its own time limit.
# usage: tools/r04_final.sh [A|B]   (A: suite, smoke, bench lines; B: the rest;
# none: both -- longer than one gpurun call allows)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r04final}
mkdir -p "$OUT"
export TMPDIR=/tmp
s() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name"; exit $rc; fi
  if grep -q -E "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "$OUT/$name.log"; then
    echo "STOP after $name (device fault)"; exit 3
  fi
}
PART=${1:-AB}
if [[ $PART == *A* ]]; then
s pytest 900 python3 -u -m pytest $R/tests -m gpu -v --timeout 300 --timeout-method thread
s smoke 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')"
s bench 400 python3 $R/bench.py
s bench_torchrun 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 $R/bench.py --gpus 1 --no-cpu-baseline
fi
if [[ $PART == *B* ]]; then
s c3 200 python3 $R/bench.py --workload config3 --no-cpu-baseline
s c4 400 python3 $R/bench.py --workload config4 --no-cpu-baseline
s c5 200 python3 $R/bench.py --workload config5 --no-cpu-baseline
s c5_64k 200 python3 $R/bench.py --workload config5 --frame-size 65536 --no-cpu-baseline
s fs1k 200 python3 $R/bench.py --frames 4194304 --frame-size 1024 --no-cpu-baseline
s fs256 200 python3 $R/bench.py --frames 16777216 --frame-size 256 --no-cpu-baseline
s split 200 python3 $R/bench.py --workload split --no-cpu-baseline
s index 200 python3 $R/bench.py --workload index
s accept 200 python3 $R/bench.py --workload accept
cd /tmp
s kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline
s fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
s write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
s kt_c5 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_c5" -o kt -- python3 $R/bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline
s kt_fs1k 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_fs1k" -o kt -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 10 --warmup 2 --no-cpu-baseline
s kt_fs256 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_fs256" -o kt -- python3 $R/bench.py --frames 16777216 --frame-size 256 --steps 10 --warmup 2 --no-cpu-baseline
s kt_split 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_split" -o kt -- python3 $R/bench.py --workload split --steps 10 --warmup 2 --no-cpu-baseline
cd $R
s config1 400 python3 $R/tools/config1_bench.py --out "$OUT/config1.jsonl" --reps 2
TAG=${TAG:-r04final} s dropin 300 bash $R/tools/dropin_lat.sh
fi
echo "== done $(date +%T)"
