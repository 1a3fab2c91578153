#!/bin/bash
# A/B of cfws_serialize_uniform builds (base = in-tree, others
# build/variants/libcfws_<v>.so from tools/mkvariant.sh; ENVS: extra
# name=VAR=value runs on the base build), 256 B and 512 B uniform batches of
# 4 GiB, the send's event time (serialize_execute ms), two rounds. RECV: the
# receive's bench flags (default the indexed info slot receive).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-uniform_ab}; mkdir -p "$OUT"
for r in 1 2; do
  for fs in ${SIZES:-256 512}; do
    F=$(( (4 << 30) / fs ))
    for v in base ${VARIANTS} ${ENVS}; do
      L=$PWD/coldforce_amd/libcfws.so; E=""
      case $v in
        base) ;;
        *=*) E=${v#*=}; ;;
        *) L=$PWD/build/variants/libcfws_$v.so ;;
      esac
      tag=${v%%=*}
      env CFWS_LIB=$L $E timeout -k 10 200 python3 bench.py --frames $F --frame-size $fs --send uniform \
          ${RECV:---recv-slots --recv-info} --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/fs${fs}_${tag}_r$r.json" 2> "$OUT/fs${fs}_${tag}_r$r.err" \
          || { echo "fs$fs $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/fs${fs}_${tag}_r$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('fs${fs}', '$tag', 'r$r', d['verified'], k['serialize_execute']['ms'], k['deserialize_execute']['ms'])"
    done
  done
done
