cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_rep
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_pipeline.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02_rep/run$i.txt 2>&1
  rc=$?
  echo "run $i rc $rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
