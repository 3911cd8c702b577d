#!/bin/bash
# PC sampling of the render kernel (debug-info build of the same sources), one
# scene per run: where the waves' issue slots and stalls go, per instruction.
# usage: tools/gpu_pcsamp.sh ROUND SCENE [SPP] [METHOD]
set -o pipefail
R=${1:-r03}; SC=${2:-c2}; SPP=${3:-32}; M=${4:-stochastic}
OUT=gpurun_out/$R/pcs_$SC
mkdir -p $OUT
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1 || { echo "rocprofv3 -L failed"; tail -5 $OUT/list.txt; }
grep -i -A12 "pc.sampl" $OUT/list.txt | head -40
if [ "$M" = stochastic ]; then
  PCS="--pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval ${PCS_INTERVAL:-65536}"
else
  PCS="--pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-100}"
fi
FSAMD_GPU_LIB=$PWD/$P/libfsgpu_dbg.so timeout -s KILL 240 rocprofv3 $PCS --kernel-trace --output-format csv -d $OUT/run -o pcs -- python3 tools/perf_ab.py default $SC $SPP 1 > $OUT/run.out 2> $OUT/run.err || { echo "pc sampling run failed"; tail -20 $OUT/run.err; exit 1; }
cat $OUT/run.out
find $OUT/run -type f | head
for f in $(find $OUT/run -name "*pc_sampling*.csv"); do gzip -k $f; ls -la $f.gz; done
