set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_idx; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_index.py tests/test_h2.py -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload index --no-cpu-baseline > $OUT/new_$r.json 2>/dev/null || exit 1
  CFWS_LIB=$PWD/build/variants/libcfws_idxold.so timeout -k 10 200 python bench.py --workload index --no-cpu-baseline > $OUT/old_$r.json 2>/dev/null || exit 1
done
