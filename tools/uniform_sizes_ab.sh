#!/bin/bash
# send A/B over sizes: base (in-tree) vs build/variants/libcfws_$V.so, uniform send, packed receive
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-absz}; mkdir -p $OUT
for r in 1 2; do for fs in ${SIZES:-4096 1024 256}; do F=$(( (4 << 30) / fs )); for v in base $V; do
  L=$PWD/coldforce_amd/libcfws.so; [ $v = base ] || L=$PWD/build/variants/libcfws_$v.so
  CFWS_LIB=$L timeout -k 10 300 python3 bench.py --frames $F --frame-size $fs --send uniform --no-cpu-baseline --steps 10 --warmup 3 > $OUT/fs${fs}_${v}_r$r.json 2> $OUT/fs${fs}_${v}_r$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/fs${fs}_${v}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('fs$fs', '$v', 'r$r', d['verified'], k['serialize_execute']['ms'])"
done; done; done
