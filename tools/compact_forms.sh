#!/bin/bash
# The small-frame step in its descriptor forms and its compact forms
# (cfws_serialize_uniform send, cfws_deserialize_slots_info receive), bench
# lines and a rocprofv3 kernel-stats pass of each; DESIGN.md section 9.
#   TAG=<dir under gpurun_out>  SIZES="256 512"  (frames = 4 GiB / size)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-compact}
mkdir -p "$OUT"
export TMPDIR=/tmp
for fs in ${SIZES:-256 512}; do
  F=$(( (4 << 30) / fs ))
  for form in "desc:--recv-slots" "compact:--recv-slots --send uniform --recv-info"; do
    name=${form%%:*}; flags=${form#*:}
    timeout -k 10 300 python3 bench.py --frames $F --frame-size $fs $flags --no-cpu-baseline --steps 20 --warmup 5 \
        > "$OUT/fs${fs}_$name.json" 2> "$OUT/fs${fs}_$name.err" || exit 1
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fs${fs}_$name" \
        -o kt -- python3 $R/bench.py --frames $F --frame-size $fs $flags --no-cpu-baseline --steps 10 --warmup 2 \
        > "$OUT/prof_fs${fs}_$name.log" 2>&1) || exit 1
    echo "fs=$fs $name done"
  done
done
