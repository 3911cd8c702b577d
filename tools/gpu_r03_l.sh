#!/bin/bash
# Round 3: mesh-root cull as straight-line masks, with hoisted segment slopes, and (measurement only) without the exact fallback.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
L="$P/libfsgpu.so $P/libfsgpu_bf.so $P/libfsgpu_bfh.so $P/libfsgpu_bfh_noex.so"
AB_TIMEOUT=200 timeout -k 10 900 bash tools/lib_ab.sh "$L" c2,c3,c4 256 2 > gpurun_out/r03/ab_root_bf.log 2>&1 || { tail gpurun_out/r03/ab_meas_bounds.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_root_bf.log
