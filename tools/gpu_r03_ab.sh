#!/bin/bash
# Round 3, final build: phase split (profiling build -DFS_PHASE_PROF) of C4, C2, C3.
set -o pipefail
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_prof.py c4,c2,c3 64 > gpurun_out/r03c/phase.log 2>&1 || { tail gpurun_out/r03c/phase.log; exit 1; }
grep -E "==|render|fs phase|fs small|fs trips" gpurun_out/r03c/phase.log
