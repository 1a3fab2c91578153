set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/s3a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 &&
timeout -k 10 300 python bench_e2e.py --workload config2 > $O/e2e_base.json 2> $O/e2e_base.err &&
CFWS_LIB=$PWD/build/variants/libcfws_a16.so timeout -k 10 300 python bench_e2e.py --workload config2 > $O/e2e_a16.json 2> $O/e2e_a16.err &&
CFWS_PIPELINE_D2H=dma timeout -k 10 300 python bench_e2e.py --workload config2 > $O/e2e_dma.json 2> $O/e2e_dma.err &&
timeout -k 10 300 python bench_e2e.py --workload config2 > $O/e2e_base2.json 2> $O/e2e_base2.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --workload config3 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --workload config3 > $O/bench_c3_torchrun.json 2> $O/bench_c3_torchrun.err
echo "exit $?"
