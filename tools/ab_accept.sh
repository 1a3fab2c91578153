#!/bin/bash
# ws_accept_kernel variants (build/variants: accold = the previous form,
# arith = base64 characters by arithmetic), parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_acc; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_handshake.py -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for v in base ${VARIANTS:-accold}; do
    if [ $v = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
    CFWS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload accept --no-cpu-baseline > $OUT/${v}_$r.json 2>/dev/null || exit 1
  done
done
