#!/bin/bash
# The round-end evidence in one GPU-box session: GPU parity suite, smoke,
# the default bench line (with the CPU baseline), the bench through
# torch.distributed.run at world size 1 (the driver's N>1 launch path),
# rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE passes.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 &&
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_torchrun.json" 2> "$OUT/bench_torchrun.err" &&
TAG=${TAG:-round}/prof bash tools/profile.sh > "$OUT/profile.txt" 2>&1
rc=$?
echo "exit $rc"
exit $rc
