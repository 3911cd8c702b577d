#!/bin/bash
# Round 3: C3 bisection over this round's commits and flags (same box, alternating processes).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
L="$P/libfsgpu_r2.so $P/libfsgpu_0567828.so $P/libfsgpu_d0f682a.so $P/libfsgpu_ff45f24.so $P/libfsgpu.so $P/libfsgpu_noROOT_PAIRS.so $P/libfsgpu_noRAD_XYZ.so"
AB_TIMEOUT=200 timeout -k 10 1000 bash tools/lib_ab.sh "$L" c3 1024 2 > gpurun_out/r03/ab_c3_bisect.log 2>&1 || { tail gpurun_out/r03/ab_c3_bisect.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_c3_bisect.log
