#!/bin/bash
# A/B of environment settings: ENVS="A=1 B=2;A=3" (';'-separated sets), 2 rounds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-envab}
mkdir -p "$OUT"
IFS=';' read -ra SETS <<< "${ENVS:-X=0}"
for round in 1 2; do
  i=0
  for e in "${SETS[@]}"; do
    name=$(echo "$e" | tr ' =' '_-')
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --workload ${WL:-config2} $ARGS \
        > "$OUT/${name}_r$round.json" 2> "$OUT/${name}_r$round.err" || { echo "set $e failed"; exit 1; }
    i=$((i+1))
  done
done
echo done
