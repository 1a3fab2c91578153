set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-ab_k}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest.txt 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then lib=$R/coldforce_amd/libcfws.so; else lib=$R/build/variants/libcfws_$v.so; fi
  for w in ${WORKLOADS:-config2 config3}; do
    CFWS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v/$w -o kt -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload $w > $OUT/$v.$w.log 2>&1 || exit 1
  done
done
echo done
