#!/bin/bash
# The one GPU-box runner (run from the repo root under gpurun). Every step runs
# under its own time limit; the first failing step ends the run.
#
# usage: bash tools/gpu_run.sh ROUND STEP [STEP ...]
#   tests[:KEXPR]                pytest -m gpu [-k KEXPR] (log + parity records in gpurun_out/ROUND)
#   smoke                        __graft_entry__.smoke()
#   bench:SCENE[:WxH[:STEPS]]    one bench.py line -> bench_SCENE_WxH.json (C4 1080p adds the CPU baseline)
#   prof[:SCENE]                 rocprofv3 --kernel-trace --stats of the bench command -> prof_SCENE/
#   flips:SCENE[:WxH[:SPP]]      tools/flip_hunt.py: GPU frame against the oracle, every differing pixel
#   sweep[:SCENES]               tools/spp_sweep.py: one launch's trace time against its samples
#   pmc:SCENE:WxH:SPP[:STEPS]    PMC passes (one counter group each) + tools/pmc_summary.py
#                                -> pmc_SCENE_WxH.json, stamped with the code object's digest
#   ab:VARIANTS:SCENES:SPP:ROUNDS   tools/perf_ab.py (fs_options A/B in one process)
#   libab:LIBS:SCENES:SPP:ROUNDS    alternating processes over in-tree builds (space-separated .so names)
#   wt[:SCENES[:SPPS]]           per-wave end/drain times of the trace kernel (needs libfsgpu_wt.so)
#   dropinlib:LIB:SCENE[:FRAMES[:DEPTH]]  the same window loop on an A/B build of libfsgpu.so
#   dropin:SCENE:FRAMES[:DEPTHS]  examples/dropin_rate (the reference's window loop) at each lookahead depth
#                                ("0 1 2"; default the library's), then a kernel + copy trace of the default
#   phase:SCENES:SPP             per-phase cycle split (needs the in-tree libfsgpu_prof.so)
#   lib:NAME                     the steps after it load final-stage-path-tracer-2-0_amd/NAME (an A/B build)
#                                through FSAMD_GPU_LIB; "lib:" alone returns to the product libfsgpu.so
#   bench:SCENE:WxH:STEPS:SPP    as bench, with a shorter spp (A/B counts)
set -o pipefail
R=$1
shift
OUT=gpurun_out/$R
mkdir -p $OUT
export TMPDIR=/tmp
fail() { echo "step failed (rc $2): $1"; [ -n "$3" ] && tail -25 "$3"; exit 1; }

for step in "$@"; do
  IFS=: read -r name a1 a2 a3 a4 <<< "$step"
  echo "== $step ($(date +%T))"
  case $name in
    lib)
      if [ -n "$a1" ]; then export FSAMD_GPU_LIB=$PWD/final-stage-path-tracer-2-0_amd/$a1; else unset FSAMD_GPU_LIB; fi
      echo "FSAMD_GPU_LIB=${FSAMD_GPU_LIB:-}" ;;
    tests)
      rm -f gpurun_out/parity_records.jsonl
      log=$OUT/pytest_gpu$([ -n "${FSAMD_GPU_LIB:-}" ] && basename ${FSAMD_GPU_LIB%.so} | sed 's/^/_/').log
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${a1:+-k "$a1"} \
        > $log 2>&1 || fail "$step" $? $log
      [ -f gpurun_out/parity_records.jsonl ] && mv gpurun_out/parity_records.jsonl $OUT/
      tail -2 $log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || fail "$step" $? $OUT/smoke.log
      tail -2 $OUT/smoke.log ;;
    bench)
      sc=${a1:-c4}; wh=${a2:-1920x1080}; w=${wh%x*}; h=${wh#*x}; st=${a3:-3}; spp=${a4:-1024}
      cpu=--no-cpu; [ "$sc$wh$spp" = c41920x10801024 ] && [ -z "${FSAMD_GPU_LIB:-}" ] && cpu=
      f=$OUT/bench_${sc}_${wh}$([ "$spp" = 1024 ] || echo "_$spp")$([ -n "${FSAMD_GPU_LIB:-}" ] && basename ${FSAMD_GPU_LIB%.so} | sed 's/^/_/')
      timeout -k 10 600 python bench.py --scene $sc --width $w --height $h --steps $st --spp $spp $cpu > $f.json \
        2> $f.err || fail "$step" $? $f.err
      cut -c1-220 $f.json ;;
    prof)
      sc=${a1:-c4}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$sc -o trace -- \
        python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu > $OUT/prof_$sc.json 2> $OUT/prof_$sc.err \
        || fail "$step" $? $OUT/prof_$sc.err
      find $OUT/prof_$sc -name "*kernel_stats.csv" -exec cut -c1-160 {} \; ;;
    pmc)
      sc=$a1; wh=$a2; w=${wh%x*}; h=${wh#*x}; spp=$a3; pst=${a4:-1}; pwu=0; [ "$pst" -gt 1 ] && pwu=2
      d=$OUT/pmc_${sc}_${wh}$([ "$spp" -lt 64 ] && echo "_$spp")
      mkdir -p $d
      cmd="python3 bench.py --scene $sc --steps $pst --warmup $pwu --spp $spp --no-cpu --width $w --height $h"
      i=0
      for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH" \
                 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
                 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
                 "GRBM_GUI_ACTIVE GRBM_COUNT"; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $d/p$i -o pmc -- $cmd \
          > $d/p$i.out 2> $d/p$i.err || fail "$step pass $i" $? $d/p$i.err
      done
      kern=$(python3 -c "import json; print([json.loads(l) for l in open('$d/p1.out') if l.startswith('{')][-1]['roofline']['kernel'])") \
        || fail "$step" $?
      # counters are averaged per dispatch: normalise by the samples of one launch (the render may take several)
      lspp=$(python3 -c "import json; print([json.loads(l) for l in open('$d/p1.out') if l.startswith('{')][-1]['roofline']['spp_per_launch'])") \
        || fail "$step" $?
      python3 tools/pmc_summary.py $d "$kern" $d.json "$sc ${wh} x $spp spp in launches of $lspp spp" \
        $((w * h * lspp)) > $d/summary.log 2>&1 || fail "$step" $? $d/summary.log
      grep -E "hbm_bytes_per_sample|valu_lane_util|wait_any|valu_issue|code_object" $d.json ;;
    flips)
      sc=$a1; wh=${a2:-1920x1080}; w=${wh%x*}; h=${wh#*x}; spp=${a3:-4}
      timeout -k 10 900 python3 tools/flip_hunt.py $sc $w $h $spp $OUT/flips_${sc}_${wh}x${spp}.json \
        > $OUT/flips_${sc}_${wh}x${spp}.log 2>&1 || fail "$step" $? $OUT/flips_${sc}_${wh}x${spp}.log
      head -3 $OUT/flips_${sc}_${wh}x${spp}.log ;;
    sweep)
      timeout -k 10 600 python3 tools/spp_sweep.py ${a1:-c4,c2} > $OUT/spp_sweep.log 2>&1 || fail "$step" $? $OUT/spp_sweep.log
      cat $OUT/spp_sweep.log ;;
    ab)
      log=$OUT/ab_$(date +%H%M%S).log
      timeout -k 10 900 python tools/perf_ab.py "$a1" "$a2" ${a3:-256} ${a4:-2} > $log 2>&1 || fail "$step" $? $log
      grep -E "variant|differs|md5" $log ;;
    libab)
      log=$OUT/libab_$(date +%H%M%S).log
      for i in $(seq 1 ${a4:-2}); do
        for L in $a1; do
          echo "== $L" >> $log
          PERF_AB_HASH=1 FSAMD_GPU_LIB=$PWD/final-stage-path-tracer-2-0_amd/$L timeout -k 10 300 \
            python tools/perf_ab.py default "$a2" ${a3:-256} 1 >> $log 2>&1 || fail "$step" $? $log
        done
      done
      grep -E "^==|variant|md5" $log ;;
    dropinlib)
      # the window loop on an A/B build: its libfsgpu.so (with the product libfshost.so) first on
      # the library path (the examples' RUNPATH yields to LD_LIBRARY_PATH)
      lib=$a1; sc=${a2:-c4}; n=${a3:-256}
      d=/tmp/fs_ablib_${lib%.so}; mkdir -p $d
      cp final-stage-path-tracer-2-0_amd/$lib $d/libfsgpu.so && cp final-stage-path-tracer-2-0_amd/libfshost.so $d/ \
        || fail "$step" $?
      p=$(python3 -c "import sys; sys.path.insert(0, 'final-stage-path-tracer-2-0_amd'); import scenes; print(scenes.write('$sc', '/tmp/fs_scenes/$sc'))") \
        || fail "$step" $?
      LD_LIBRARY_PATH=$d timeout -k 10 300 ./examples/dropin_rate $p 1920 1080 $n ${a4:-} >> $OUT/dropin_${sc}_${lib%.so}.json \
        2> $OUT/dropin_${sc}_${lib%.so}.err || fail "$step" $? $OUT/dropin_${sc}_${lib%.so}.err
      tail -1 $OUT/dropin_${sc}_${lib%.so}.json ;;
    dropin)
      # the reference's window loop through the C++ mirror (examples/dropin_rate), then the same
      # loop under a kernel + memory-copy trace (per-frame split: trace, fold, copies, gaps)
      sc=${a1:-c4}; n=${a2:-256}; la=${a3:-}
      p=$(python3 -c "import sys; sys.path.insert(0, 'final-stage-path-tracer-2-0_amd'); import scenes; print(scenes.write('$sc', '/tmp/fs_scenes/$sc'))") \
        || fail "$step" $?
      for d in ${la:-default}; do
        [ "$d" = default ] && d=
        timeout -k 10 300 ./examples/dropin_rate $p 1920 1080 $n $d >> $OUT/dropin_${sc}_1920x1080.json \
          2> $OUT/dropin_$sc.err || fail "$step" $? $OUT/dropin_$sc.err
      done
      cat $OUT/dropin_${sc}_1920x1080.json
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
        -d $OUT/dropin_prof_$sc -o trace -- ./examples/dropin_rate $p 1920 1080 64 ${la##* } > $OUT/dropin_prof_$sc.json \
        2> $OUT/dropin_prof_$sc.err || fail "$step" $? $OUT/dropin_prof_$sc.err
      python3 tools/dropin_split.py $OUT/dropin_prof_$sc > $OUT/dropin_split_$sc.log 2>&1 || fail "$step" $? $OUT/dropin_split_$sc.log
      cat $OUT/dropin_split_$sc.log ;;
    wt)
      FSAMD_GPU_LIB=$PWD/final-stage-path-tracer-2-0_amd/libfsgpu_wt.so timeout -k 10 600 \
        python tools/wave_times.py ${a1:-c4,c2} ${a2:-1,2,16} > $OUT/wave_times.log 2>&1 || fail "$step" $? $OUT/wave_times.log
      grep -E "==|waves" $OUT/wave_times.log ;;
    phase)
      FSAMD_GPU_LIB=$PWD/final-stage-path-tracer-2-0_amd/libfsgpu_prof.so timeout -k 10 600 \
        python tools/phase_prof.py "$a1" ${a2:-64} > $OUT/phase.log 2>&1 || fail "$step" $? $OUT/phase.log
      grep -E "==|phase|trips" $OUT/phase.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done ($(date +%T))"
