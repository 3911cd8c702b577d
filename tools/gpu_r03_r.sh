#!/bin/bash
# Round 3: phase split of the current build (profiling build).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_prof.py c4,c2,c3 64 > gpurun_out/r03/phase2.log 2>&1 || { tail gpurun_out/r03/phase2.log; exit 1; }
grep -E "==|render|fs " gpurun_out/r03/phase2.log
