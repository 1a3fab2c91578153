set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02_gridgap
mkdir -p $OUT
for g in 0 65536 16384; do
  CFWS_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/g$g -o kt -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/g$g.log 2>&1 || exit 1
done
