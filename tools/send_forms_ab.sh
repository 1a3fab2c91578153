#!/bin/bash
# The uniform send (cfws_serialize_uniform) against the descriptor send
# (cfws_serialize_batch: plan + execute; the event time is the execute's)
# across frame sizes, alternating on one box, packed receive; prints the
# send's event ms and the step ms per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sendforms}; mkdir -p $OUT
for r in 1 2; do for fs in ${SIZES:-512 1024 4096 65536}; do F=$(( (4 << 30) / fs )); for form in uniform batch; do
  timeout -k 10 300 python3 bench.py --frames $F --frame-size $fs --send $form --no-cpu-baseline --steps 10 \
      --warmup 3 > $OUT/fs${fs}_${form}_r$r.json 2> $OUT/fs${fs}_${form}_r$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/fs${fs}_${form}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('fs$fs', '$form', 'r$r', d['verified'], k['serialize_execute']['ms'], d['ms_per_step'])"
done; done; done
