#!/bin/bash
# Round 3: upper bounds from measurement-only builds (root culls, divisions, backward pass).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
L="$P/libfsgpu.so $P/libfsgpu_mroot.so $P/libfsgpu_mdiv.so $P/libfsgpu_munw.so"
AB_TIMEOUT=200 timeout -k 10 900 bash tools/lib_ab.sh "$L" c2,c3,c4 256 2 > gpurun_out/r03/ab_meas_bounds.log 2>&1 || { tail gpurun_out/r03/ab_meas_bounds.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_meas_bounds.log
