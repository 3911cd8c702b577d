#!/bin/bash
# Round 3: the device code object built for gfx950:xnack- (no XNACK replay assumed)
# against the product build (xnack any); frames must be identical.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
PERF_AB_HASH=1 AB_TIMEOUT=300 timeout -k 10 900 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_xnm.so" c2,c3,c4 256 3 > gpurun_out/r03/ab_xnack.log 2>&1 || { tail gpurun_out/r03/ab_xnack.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_xnack.log
