#!/bin/bash
# cfws_serialize_uniform under environment knobs (ENVS: name=VAR=value ...)
# across frame sizes (SIZES), uniform send + packed receive, two rounds; prints
# the send's event time per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-uenv}; mkdir -p $OUT
for r in 1 2; do for fs in ${SIZES:-4096 1024}; do F=$(( (4 << 30) / fs )); for v in base ${ENVS}; do
  tag=${v%%=*}; E=""; [ $v = base ] || E=${v#*=}
  env $E timeout -k 10 300 python3 bench.py --frames $F --frame-size $fs --send uniform --no-cpu-baseline --steps 10 --warmup 3 > $OUT/fs${fs}_${tag}_r$r.json 2> $OUT/fs${fs}_${tag}_r$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/fs${fs}_${tag}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('fs$fs', '$tag', 'r$r', d['verified'], k['serialize_execute']['ms'])"
done; done; done
