set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_c3split; mkdir -p $OUT
for r in 1 2; do
for v in base n1; do
  if [ "$v" = base ]; then lib=coldforce_amd/libcfws.so; else lib=build/variants/libcfws_$v.so; fi
  for sp in 0 1; do
    CFWS_EDGE_SPLIT=$sp CFWS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --workload config3 > $OUT/${v}_split${sp}_r$r.json 2>/dev/null || exit 1
  done
done
done
