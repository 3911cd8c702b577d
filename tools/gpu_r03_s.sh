#!/bin/bash
# Round 3: phase split of the current build, then a re-sweep of the parking and small-mesh settings.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_prof.py c4,c2,c3 64 > gpurun_out/r03/phase2.log 2>&1 || { tail gpurun_out/r03/phase2.log; exit 1; }
grep -E "==|render|fs phase|fs small|fs trips" gpurun_out/r03/phase2.log
timeout -k 10 600 python tools/perf_ab.py "default,park_lanes=12,park_lanes=14,park_lanes=16,park_lanes=12@park_lanes_small=8" c3,c4 256 2 > gpurun_out/r03/ab_park_sweep.log 2>&1 || { tail gpurun_out/r03/ab_park_sweep.log; exit 1; }
cat gpurun_out/r03/ab_park_sweep.log
P=final-stage-path-tracer-2-0_amd
PERF_AB_HASH=1 AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu_cur.so $P/libfsgpu_pipe.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_unwind_pipe.log 2>&1 || { tail gpurun_out/r03/ab_unwind_pipe.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_unwind_pipe.log
