#!/bin/bash
# Round 3: this round's build against round 2's final build (same box, alternating processes).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 800 bash tools/lib_ab.sh "$P/libfsgpu_r2.so $P/libfsgpu.so" c2,c3,c4 1024 2 > gpurun_out/r03/ab_r2_vs_r3.log 2>&1 || { tail gpurun_out/r03/ab_r2_vs_r3.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_r2_vs_r3.log
