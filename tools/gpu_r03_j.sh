#!/bin/bash
# Round 3: park_entry / root-pair code A/B against round 2 (same box, alternating processes).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
L="$P/libfsgpu_r2.so $P/libfsgpu.so $P/libfsgpu_noPE.so $P/libfsgpu_noPE_noRP.so $P/libfsgpu_noROOT_PAIRS.so"
AB_TIMEOUT=200 timeout -k 10 1000 bash tools/lib_ab.sh "$L" c3,c4 1024 2 > gpurun_out/r03/ab_pe.log 2>&1 || { tail gpurun_out/r03/ab_pe.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_pe.log
