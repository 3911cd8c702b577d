#!/bin/bash
# PMC passes on the bench workload (reduced spp), one counter group per pass.
set -o pipefail
R=${1:-r01}; SPP=${2:-512}  # 512 spp = one launch of 8 sample groups of 64, the bench launch shape
mkdir -p gpurun_out/$R/pmc
export TMPDIR=/tmp
CMD="python3 bench.py --steps 1 --warmup 0 --spp $SPP --no-cpu"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$R/pmc/p$i -o pmc -- $CMD > gpurun_out/$R/pmc/p$i.out 2> gpurun_out/$R/pmc/p$i.err || { echo "pass $i failed"; tail -5 gpurun_out/$R/pmc/p$i.err; exit 1; }
done
ls gpurun_out/$R/pmc/*/
