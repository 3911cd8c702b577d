#!/bin/bash
# PMC passes on a bench workload (reduced spp), one counter group per pass.
# usage: tools/gpu_pmc.sh ROUND [SPP] [WIDTH HEIGHT] [SCENE]
set -o pipefail
R=${1:-r01}; SPP=${2:-512}  # 512 spp = one launch of 32 sample groups of 16, the bench launch shape
W=${3:-1920}; H=${4:-1080}; SC=${5:-c4}
OUT=gpurun_out/$R/pmc_${SC}$([ "$W" = 1920 ] || echo "_${W}x${H}")
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --scene $SC --steps 1 --warmup 0 --spp $SPP --no-cpu --width $W --height $H"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" ${PMC_EXTRA:-}; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- $CMD > $OUT/p$i.out 2> $OUT/p$i.err || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.err; exit 1; }
done
ls $OUT/*/
