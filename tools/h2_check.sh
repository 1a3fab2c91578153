set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/h2a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_h2.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --workload config5 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --workload config5 --frame-size 65536 > $O/c5_64k.json 2> $O/c5_64k.err &&
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o c5 -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --workload config5 --steps 10 --warmup 2 ) > $O/prof.txt 2>&1
echo "exit $?"
