#!/bin/bash
# Round 3, call 5: 7-wave parked-walk kernel A/B, then PMC summaries of C4, C2, C3.
set -o pipefail
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_s7.so" c3,c4 256 2 > gpurun_out/r03/ab_susp7.log 2>&1 || { tail gpurun_out/r03/ab_susp7.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_susp7.log
for sc in c4 c2 c3; do
  bash tools/gpu_pmc.sh r03 512 1920 1080 $sc > gpurun_out/r03/pmc_$sc.log 2>&1 || { tail gpurun_out/r03/pmc_$sc.log; exit 1; }
  echo "pmc $sc done"
done
