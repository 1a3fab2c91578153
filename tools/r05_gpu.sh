#!/bin/bash
# Round-5 GPU session: parity suite, benches, kernel stats, PMC passes.
# Each GPU step has its own time limit; a fault, abort, segfault or time
# limit (rc 124/134/137/139 or > 128) ends the script; a plain test failure
# (rc 1) does not.
# usage: tools/r05_gpu.sh TAG STEP...   (steps: the case labels below, e.g.
#   pytest smoke bench digests guard slots fs256 fs256s fs1k fs1ks kstats
#   kstats_fs256s c5cpu e2e ab_plan ab_slots256 envab_sub2 pmc_sq_send ...;
#   VARIANTS / V256 / VPLAN / VF / VBIG pick build/variants for the ab_ steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  # a device fault reported as a Python exception (rc 1): stop too
  if grep -q -E "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "$OUT/$name.log"; then
    echo "STOP after $name (device fault)"; exit 3
  fi
  return 0
}
pmc() {  # name workload-args... ; counters in $C
  step "pmc_$1" 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$1" -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "${@:2}"
}
for s in "$@"; do
  case $s in
    pytest) step pytest 900 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    guard) step guard 600 python3 -u -m pytest $R/tests/test_gpu_guard.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    digests) step digests 600 python3 -u -m pytest $R/tests/test_gpu_batch.py -m gpu -x -v -k small_frame_reference_digests --timeout 300 --timeout-method thread ;;
    pyk) step pyk_$(echo "$K" | tr -c 'a-zA-Z0-9' _ | cut -c1-60) 900 python3 -u -m pytest $(for f in $TESTS; do echo $R/tests/$f; done) -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread ;;
    pytest_sub) step pytest_sub 900 python3 -u -m pytest $(for f in $TESTS; do echo $R/tests/$f; done) -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) step bench 400 python3 $R/bench.py ;;
    split) step split 200 python3 $R/bench.py --workload split --no-cpu-baseline ;;
    c5) step c5 200 python3 $R/bench.py --workload config5 --no-cpu-baseline ;;
    e2e) for w in config2 config3 config5; do step e2e_$w 400 python3 $R/bench_e2e.py --workload $w; done
         step e2e_config5_64k 400 python3 $R/bench_e2e.py --workload config5 --frame-size 65536 ;;
    c5cpu) step c5cpu 300 python3 $R/bench.py --workload config5 ;;
    prof_c5) step prof_c5 600 env TAG=$TAG/prof_c5 ARGS="--workload config5" bash $R/tools/profile.sh ;;
    c3) step c3 200 python3 $R/bench.py --workload config3 --no-cpu-baseline ;;
    slots) step slots 600 python3 -u -m pytest $R/tests/test_gpu_slots.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    fs256s) step fs256s 200 python3 $R/bench.py --frames 16777216 --frame-size 256 --no-cpu-baseline --recv-slots ;;
    fs1ks) step fs1ks 200 python3 $R/bench.py --frames 4194304 --frame-size 1024 --no-cpu-baseline --recv-slots ;;
    fs512s) step fs512s 200 python3 $R/bench.py --frames 8388608 --frame-size 512 --no-cpu-baseline --recv-slots ;;
    fs512) step fs512 200 python3 $R/bench.py --frames 8388608 --frame-size 512 --no-cpu-baseline ;;
    kstats_fs256s) step kstats_fs256s 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_fs256s" -o ks -- python3 $R/bench.py --frames 16777216 --frame-size 256 --steps 10 --warmup 3 --no-cpu-baseline --recv-slots ;;
    prof_fs256s) step prof_fs256s 400 env TAG=$TAG/prof_fs256s ARGS="--frames 16777216 --frame-size 256 --recv-slots" bash $R/tools/profile.sh ;;
    prof_fs256s_gen) step prof_fs256s_gen 400 env CFWS_SLOTS_WINDOW=0 TAG=$TAG/prof_fs256s_gen ARGS="--frames 16777216 --frame-size 256 --recv-slots" bash $R/tools/profile.sh ;;
    fs256s_gen) step fs256s_gen 200 env CFWS_SLOTS_WINDOW=0 python3 $R/bench.py --frames 16777216 --frame-size 256 --no-cpu-baseline --recv-slots ;;
    fs512s_gen) step fs512s_gen 200 env CFWS_SLOTS_WINDOW=0 python3 $R/bench.py --frames 8388608 --frame-size 512 --no-cpu-baseline --recv-slots ;;
    slotab) step slotab 600 env TAG=$TAG/slotab ENVS="X=0;CFWS_SLOT_GRID=2048;CFWS_SLOT_GRID=4096" ARGS="--frames 16777216 --frame-size 256 --recv-slots" bash $R/tools/envab.sh ;;
    ab_slots256) step ab_slots256 900 env TAG=$TAG/ab_slots256 VARIANTS="${V256:-base}" ARGS="--frames 16777216 --frame-size 256 --recv-slots" bash $R/tools/ab.sh ;;
    ab_slots512) step ab_slots512 900 env TAG=$TAG/ab_slots512 VARIANTS="${V512:-base}" ARGS="--frames 8388608 --frame-size 512 --recv-slots" bash $R/tools/ab.sh ;;
    ab_slots1k) step ab_slots1k 900 env TAG=$TAG/ab_slots1k VARIANTS="${V1K:-base}" ARGS="--frames 4194304 --frame-size 1024 --recv-slots" bash $R/tools/ab.sh ;;
    fs2ks) step fs2ks 200 python3 $R/bench.py --frames 2097152 --frame-size 2048 --no-cpu-baseline --recv-slots ;;
    fs1500s) step fs1500s 200 python3 $R/bench.py --frames 2796202 --frame-size 1536 --no-cpu-baseline --recv-slots ;;
    fs3ks) step fs3ks 200 python3 $R/bench.py --frames 1398101 --frame-size 3072 --no-cpu-baseline --recv-slots ;;
    fs4ks) step fs4ks 200 python3 $R/bench.py --frames 1048576 --frame-size 4096 --no-cpu-baseline --recv-slots ;;
    fs8ks) step fs8ks 200 python3 $R/bench.py --frames 524288 --frame-size 8192 --no-cpu-baseline --recv-slots ;;
    fs4k) step fs4k 200 python3 $R/bench.py --frames 1048576 --frame-size 4096 --no-cpu-baseline ;;
    fs8k) step fs8k 200 python3 $R/bench.py --frames 524288 --frame-size 8192 --no-cpu-baseline ;;
    ab_slots2k) step ab_slots2k 900 env TAG=$TAG/ab_slots2k VARIANTS="${V2K:-base}" ARGS="--frames 2097152 --frame-size 2016 --recv-slots" bash $R/tools/ab.sh ;;
    ab_slots3k) step ab_slots3k 900 env TAG=$TAG/ab_slots3k VARIANTS="${V3K:-base}" ARGS="--frames 1398101 --frame-size 3072 --recv-slots" bash $R/tools/ab.sh ;;
    smoke) step smoke 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    kstats_fs1ks) step kstats_fs1ks 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_fs1ks" -o ks -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 10 --warmup 3 --no-cpu-baseline --recv-slots ;;
    ab_wide) for w in "16777216 256" "4194304 1024" "1398101 3072"; do set -- $w; step ab_wide_$2 900 env TAG=$TAG/ab_wide_$2 VARIANTS="base wide" ARGS="--frames $1 --frame-size $2" bash $R/tools/ab.sh; done ;;
    ab_plan) for w in "16777216 256" "4194304 1024" "1398101 3072"; do set -- $w; step ab_plan_$2 900 env TAG=$TAG/ab_plan_$2 VARIANTS="${VPLAN:-base}" ARGS="--frames $1 --frame-size $2" bash $R/tools/ab.sh; done ;;
    ab_fused256) step ab_fused256 900 env TAG=$TAG/ab_fused256 VARIANTS="${VF:-base}" ARGS="--frames 16777216 --frame-size 256" bash $R/tools/ab.sh ;;
    envab_fused512) step envab_fused512 600 env TAG=$TAG/envab_fused512 ENVS="X=0;CFWS_FUSED_AVG_MAX=600" ARGS="--frames 8388608 --frame-size 512" bash $R/tools/envab.sh ;;
    envab_fused1k) step envab_fused1k 600 env TAG=$TAG/envab_fused1k ENVS="X=0;CFWS_FUSED_AVG_MAX=1100" ARGS="--frames 4194304 --frame-size 1024" bash $R/tools/envab.sh ;;
    pmc_sq_send)
      C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
      pmc sq_fs256 --frames 16777216 --frame-size 256 && pmc sq_c2 && pmc sq_fs1k --frames 4194304 --frame-size 1024 ;;
    envab_sub2) for w in "16777216 256" "8388608 512" "11184810 384" "5592405 768"; do set -- $w; step envab_sub2_$2 600 env TAG=$TAG/envab_sub2_$2 ENVS="CFWS_SLOT_SUB2_G=65;X=0;CFWS_SLOT_SUB2_G=17" ARGS="--frames $1 --frame-size $2 --recv-slots" bash $R/tools/envab.sh; done ;;
    envab_sub4) for w in "4194304 1024" "3495253 1200"; do set -- $w; step envab_sub4_$2 600 env TAG=$TAG/envab_sub4_$2 ENVS="X=0;CFWS_SLOT_SUB4_G=65" ARGS="--frames $1 --frame-size $2 --recv-slots" bash $R/tools/envab.sh; done ;;
    fs6ks) step fs6ks 200 python3 $R/bench.py --frames 699050 --frame-size 6144 --no-cpu-baseline --recv-slots ;;
    fs6k) step fs6k 200 python3 $R/bench.py --frames 699050 --frame-size 6144 --no-cpu-baseline ;;
    ab_slots_big) for w in "524288 8192" "65536 65536"; do set -- $w; step ab_slots_big_$2 900 env TAG=$TAG/ab_slots_big_$2 VARIANTS="${VBIG:-base}" ARGS="--frames $1 --frame-size $2 --recv-slots" bash $R/tools/ab.sh; done ;;
    fs256x) step fs256x 200 python3 $R/bench.py --frames 16777216 --frame-size 256 --no-cpu-baseline --recv-scatter ;;
    fs1kx) step fs1kx 200 python3 $R/bench.py --frames 4194304 --frame-size 1024 --no-cpu-baseline --recv-scatter ;;
    fs256) step fs256 200 python3 $R/bench.py --frames 16777216 --frame-size 256 --no-cpu-baseline ;;
    kstats_fs256) step kstats_fs256 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_fs256" -o ks -- python3 $R/bench.py --frames 16777216 --frame-size 256 --steps 10 --warmup 3 --no-cpu-baseline ;;
    fs2k) step fs2k 200 python3 $R/bench.py --frames 2097152 --frame-size 2048 --no-cpu-baseline ;;
    fs3k) step fs3k 200 python3 $R/bench.py --frames 1398101 --frame-size 3072 --no-cpu-baseline ;;
    fs1k) step fs1k 200 python3 $R/bench.py --frames 4194304 --frame-size 1024 --no-cpu-baseline ;;
    config1) step config1 400 python3 $R/tools/config1_bench.py --out "$OUT/config1.jsonl" --reps 2 ;;
    dropin) step dropin 400 env TAG=$TAG bash $R/tools/dropin_lat.sh ;;
    kstats) step kstats 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats" -o ks -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    kstats_c5) step kstats_c5 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_c5" -o ks -- python3 $R/bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline ;;
    kstats_fs1k) step kstats_fs1k 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_fs1k" -o ks -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 10 --warmup 3 --no-cpu-baseline ;;
    kstats_split) step kstats_split 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_split" -o ks -- python3 $R/bench.py --workload split --steps 10 --warmup 3 --no-cpu-baseline ;;
    knobs_fused) step knobs_fused 600 python3 -u -m pytest $R/tests/test_knobs.py -m gpu -x -v -k FUSED --timeout 300 --timeout-method thread ;;
    envab_fs1k) step envab_fs1k 600 env TAG=$TAG/envab_fs1k ARGS="--frames 4194304 --frame-size 1024" bash $R/tools/envab.sh ;;
    envab_fs3k) step envab_fs3k 900 env TAG=$TAG/envab_fs3k ARGS="--frames 1398101 --frame-size 3072" bash $R/tools/envab.sh ;;
    envab_fs1k2) step envab_fs1k2 900 env TAG=$TAG/envab_fs1k ARGS="--frames 4194304 --frame-size 1024" bash $R/tools/envab.sh ;;
    envab_fs2k) step envab_fs2k 900 env TAG=$TAG/envab_fs2k ARGS="--frames 2097152 --frame-size 2048" bash $R/tools/envab.sh ;;
    envab_fs4k) step envab_fs4k 900 env TAG=$TAG/envab_fs4k ARGS="--frames 1048576 --frame-size 4096" bash $R/tools/envab.sh ;;
    envab_fs8k) step envab_fs8k 900 env TAG=$TAG/envab_fs8k ARGS="--frames 524288 --frame-size 8192" bash $R/tools/envab.sh ;;
    envab_c3) step envab_c3 900 env TAG=$TAG/envab_c3 WL=config3 bash $R/tools/envab.sh ;;
    envab_fs256) step envab_fs256 600 env TAG=$TAG/envab_fs256 ARGS="--frames 16777216 --frame-size 256" bash $R/tools/envab.sh ;;
    kstats_staged) step kstats_staged 200 env CFWS_FUSED_DESER=2 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats_staged" -o ks -- python3 $R/bench.py --frames 4194304 --frame-size 1024 --steps 10 --warmup 3 --no-cpu-baseline ;;
    list) step list 60 rocprofv3 -L ;;
    prof_c2) step prof_c2 400 env TAG=$TAG/prof_c2 bash $R/tools/profile.sh ;;
    prof_fs1k) step prof_fs1k 400 env TAG=$TAG/prof_fs1k ARGS="--frames 4194304 --frame-size 1024" bash $R/tools/profile.sh ;;
    prof_fs256) step prof_fs256 400 env TAG=$TAG/prof_fs256 ARGS="--frames 16777216 --frame-size 256" bash $R/tools/profile.sh ;;
    ab) step ab 600 env TAG=$TAG/ab bash $R/tools/ab.sh ;;
    ab_fs1k) step ab_fs1k 600 env TAG=$TAG/ab_fs1k ARGS="--frames 4194304 --frame-size 1024" bash $R/tools/ab.sh ;;
    ab_fs256) step ab_fs256 600 env TAG=$TAG/ab_fs256 ARGS="--frames 16777216 --frame-size 256" bash $R/tools/ab.sh ;;
    envab) step envab 600 env TAG=$TAG/envab bash $R/tools/envab.sh ;;
    pmc_c5ab)
      for v in 1 0; do
        step pmc_c5ab_wr$v 120 env CFWS_H2_INREG=$v rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/pmc_c5ab_wr$v" -o pmc -- python3 $R/bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline
        step pmc_c5ab_sq$v 120 env CFWS_H2_INREG=$v rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_c5ab_sq$v" -o pmc -- python3 $R/bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline
      done ;;
    pmc)
      C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
      pmc sq_c2 && pmc sq_c5 --workload config5
      C="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
      pmc tcc_c2 && pmc tcc_c5 --workload config5
      C="TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
      pmc tcp_c2 && pmc tcp_c5 --workload config5 ;;
  esac
done
echo "== done $(date +%T)"
