#!/bin/bash
# Serialize vs deserialize per-frame boundary cost: deserialize with packed
# (align 1) payloads has edge chunks and boundary regions like serialize;
# CFWS_EDGE_SPLIT=1 moves the edge chunks to a launch of their own.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_asym
mkdir -p $OUT
timeout -k 10 300 python tools/layout_probe.py --reps 10 --orders SSSS,DDDD --align 16 > $OUT/a16.jsonl 2> $OUT/a16.err &&
timeout -k 10 300 python tools/layout_probe.py --reps 10 --orders SSSS,DDDD --align 1 > $OUT/a1.jsonl 2> $OUT/a1.err &&
CFWS_EDGE_SPLIT=1 timeout -k 10 300 python tools/layout_probe.py --reps 10 --orders SSSS,DDDD --align 1 > $OUT/a1_split.jsonl 2> $OUT/a1_split.err
