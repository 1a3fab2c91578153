#!/bin/bash
# ws_accept_kernel: the 24-byte-key fast form against the byte-wise message
# build (accold), parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_acc; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_handshake.py -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload accept --no-cpu-baseline > $OUT/new_$r.json 2>/dev/null || exit 1
  CFWS_LIB=$PWD/build/variants/libcfws_accold.so timeout -k 10 200 python bench.py --workload accept --no-cpu-baseline > $OUT/old_$r.json 2>/dev/null || exit 1
done
