#!/bin/bash
# Pipeline parity, then host-to-host config 2 for the in-tree library vs a
# variant (VARIANT, build/variants/libcfws_<VARIANT>.so), kernel D2H and SDMA
# D2H (CFWS_PIPELINE_D2H=dma), x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-outab}
mkdir -p "$OUT"
WL=${WL:-config2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || exit 1
CFWS_PIPELINE_D2H=dma timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_dma.txt" 2>&1 || exit 1
for r in 1 2; do
  for v in base ${VARIANT:-slotout}; do
    if [ $v = base ]; then L=$PWD/coldforce_amd/libcfws.so; else L=$PWD/build/variants/libcfws_$v.so; fi
    CFWS_LIB=$L timeout -k 10 300 python bench_e2e.py --workload $WL > "$OUT/${v}_kernel_$r.json" 2>> "$OUT/err.txt" &&
    CFWS_LIB=$L CFWS_PIPELINE_D2H=dma timeout -k 10 300 python bench_e2e.py --workload $WL > "$OUT/${v}_dma_$r.json" 2>> "$OUT/err.txt" || exit 1
  done
done
echo "exit 0"
