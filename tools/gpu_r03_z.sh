#!/bin/bash
# Round 3, final build (walk priority off): parking re-sweep, the round-end
# evidence (GPU suite, smoke, bench lines, rocprofv3 stats) and C4 PMC passes.
set -o pipefail
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
timeout -k 10 600 python tools/perf_ab.py "default,park_lanes=10,park_lanes=14,park_lanes_small=4,park_lanes_small=8" c3,c4 256 2 > gpurun_out/r03c/ab_park.log 2>&1 || { tail gpurun_out/r03c/ab_park.log; exit 1; }
grep -E "variant|differs" gpurun_out/r03c/ab_park.log
bash tools/gpu_round_check.sh r03c || exit 1
bash tools/gpu_pmc.sh r03c 512 1920 1080 c4 > gpurun_out/r03c/pmc_c4.log 2>&1 || { tail gpurun_out/r03c/pmc_c4.log; exit 1; }
echo pmc done
