#!/bin/bash
# Round 3: mesh-root cull outcomes (profiling builds of the straight-line cull, 1e-5 and error-bound margins).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=$PWD/final-stage-path-tracer-2-0_amd
timeout -k 10 300 python tools/phase_prof.py c2,c3,c4 32 > gpurun_out/r03/root_stats.log 2>&1 || { tail gpurun_out/r03/root_stats.log; exit 1; }
FSAMD_GPU_LIB=$P/libfsgpu_proft.so timeout -k 10 300 python tools/phase_prof.py c2,c3,c4 32 > gpurun_out/r03/root_stats_tol.log 2>&1 || { tail gpurun_out/r03/root_stats_tol.log; exit 1; }
grep -E "==|render|fs root" gpurun_out/r03/root_stats.log gpurun_out/r03/root_stats_tol.log
