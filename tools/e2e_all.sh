#!/bin/bash
# Pipeline parity (every host-memory kind x D2H mode), then the host-to-host
# rates of configs 2, 3, 5: mapped arenas in the default D2H mode, and torch
# pinned arenas. One GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-e2eall}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
for wl in config2 config3 config5; do
  for host in mapped torch; do
    timeout -k 10 300 python bench_e2e.py --workload $wl --host $host > "$OUT/${wl}_${host}.json" 2> "$OUT/${wl}_${host}.err" || { echo "$wl $host failed"; exit 1; }
  done
done
echo "exit 0"
