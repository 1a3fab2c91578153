#!/bin/bash
# tools/pipeline_stress.py on the in-tree build and on the round-1 store
# policy (oldpol), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_stress; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python tools/pipeline_stress.py --reps 25 > $OUT/new_$r.jsonl 2> $OUT/new_$r.err || exit 1
  CFWS_LIB=$PWD/build/variants/libcfws_oldpol.so timeout -k 10 300 python tools/pipeline_stress.py --reps 25 > $OUT/old_$r.jsonl 2> $OUT/old_$r.err || exit 1
done
