#!/bin/bash
# The multi-rank bench path on a one-GPU box: torchrun with N ranks sharing
# the GPU (CFWS_BENCH_REHEARSE=1: gloo bookkeeping collectives), every
# workload. Checks that each line is emitted, verified and reports n_gpus = N;
# the rates are not measurements (the ranks share one device).
# usage: tools/rehearse.sh [N]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-2}
OUT=gpurun_out/${TAG:-rehearse}
mkdir -p "$OUT"
export CFWS_BENCH_REHEARSE=1
port=29611
for wl in config2 config3 config5 split index accept fs1k; do
  case $wl in
    fs1k) a="--frames 4194304 --frame-size 1024" ;;
    *) a="--workload $wl" ;;
  esac
  port=$((port + 1))
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $N --steps 5 --warmup 2 --no-cpu-baseline $a > "$OUT/${wl}_n$N.log" 2>&1
  rc=$?
  echo "== $wl n=$N rc=$rc"
  grep '^{' "$OUT/${wl}_n$N.log" | tail -1 | cut -c1-220
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${wl}_n$N.log"; exit $rc; fi
done
echo done
