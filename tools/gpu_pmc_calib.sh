#!/bin/bash
# PMC counter calibration on known byte counts (tools/pmc_calib.py).
set -o pipefail
R=${1:-calib}
mkdir -p gpurun_out/$R
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$R/p$i -o pmc -- python3 tools/pmc_calib.py > gpurun_out/$R/p$i.out 2> gpurun_out/$R/p$i.err || { echo "pass $i failed"; tail -5 gpurun_out/$R/p$i.err; exit 1; }
done
