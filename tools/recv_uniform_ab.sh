#!/bin/bash
# The slot receive of a uniform batch with its index (cfws_deserialize_slots_info)
# against the implicit-stride form (cfws_deserialize_slots_uniform), both
# after the uniform send, alternating on one box (SIZES, ROUNDS); prints the
# receive's event time per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-runi}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do for fs in ${SIZES:-256 512 1024 4096}; do F=$(( (4 << 30) / fs ))
  for form in "indexed:--recv-slots --recv-info" "implicit:--recv-uniform"; do
    name=${form%%:*}; flags=${form#*:}
    timeout -k 10 300 python3 bench.py --frames $F --frame-size $fs --send uniform $flags --no-cpu-baseline \
        --steps 10 --warmup 3 > $OUT/fs${fs}_${name}_r$r.json 2> $OUT/fs${fs}_${name}_r$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/fs${fs}_${name}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('fs$fs', '$name', 'r$r', d['verified'], k['deserialize_execute']['ms'], d['ms_per_step'])"
  done
done; done
