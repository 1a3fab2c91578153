set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c15
for v in base im4096 im16384 im65535; do
  if [ $v = base ]; then L=$PWD/coldforce_amd/libcfws.so; else L=$PWD/build/variants/libcfws_$v.so; fi
  CFWS_LIB=$L timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -k "serialize or digest" --timeout 250 --timeout-method thread > gpurun_out/c15/pytest_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/c15/pytest_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
  if grep -q -E "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/c15/pytest_$v.log; then exit 3; fi
done
for fs in 2048 4096 16384 32768; do
  VARIANTS="base im4096 im16384 im65535" TAG=c15/ab_fs$fs ARGS="--frames $((4294967296 / fs)) --frame-size $fs" timeout -k 10 600 bash tools/ab.sh > gpurun_out/c15/ab_fs$fs.log 2>&1 || { echo "ab $fs failed"; exit 1; }
done
echo ok
