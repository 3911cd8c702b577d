#!/bin/bash
# Round 3, call 8: object-record header in one scalar load, A/B.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 800 bash tools/lib_ab.sh "$P/libfsgpu_head0.so $P/libfsgpu.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_objhead.log 2>&1 || { tail gpurun_out/r03/ab_objhead.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_objhead.log
