#!/bin/bash
# Round 3 (final build): PMC passes of the bench kernels (C4, C2, C3), one counter group per pass.
set -o pipefail
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
for sc in c4 c2 c3; do
  bash tools/gpu_pmc.sh r03f 512 1920 1080 $sc > gpurun_out/r03f/pmc_$sc.log 2>&1 || { tail gpurun_out/r03f/pmc_$sc.log; exit 1; }
  echo "pmc $sc done"
done
