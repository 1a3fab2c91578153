#!/bin/bash
# two_frame_region rewrite (uniform scalars) against the previous form (v1):
# GPU parity suite on the new build, then A/B on configs 2, 3 and 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_ab_twoframe
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02_ab_twoframe/pytest_gpu.txt 2>&1 &&
TAG=r02_ab_twoframe/c2 VARIANTS="base v1" WL=config2 bash tools/ab.sh &&
TAG=r02_ab_twoframe/c3 VARIANTS="base v1" WL=config3 bash tools/ab.sh &&
TAG=r02_ab_twoframe/c5 VARIANTS="base v1" WL=config5 bash tools/ab.sh
