#!/bin/bash
# general_region with lane-parallel frame loads vs the per-chunk search
# (old), with and without the send-direction write-through at 4 WG/CU (n1):
# GPU parity first, then configs 3 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_ab_general
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02_ab_general/pytest_gpu.txt 2>&1 &&
TAG=r02_ab_general/c3 VARIANTS="base old n1 n1old" WL=config3 bash tools/ab.sh &&
TAG=r02_ab_general/c2 VARIANTS="base n1" WL=config2 bash tools/ab.sh
