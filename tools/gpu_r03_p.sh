#!/bin/bash
# Round 3: lane-major HBM shading rows with the backward pass's c values prefetched (A/B, frame hashes).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp PERF_AB_HASH=1
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu_cur.so $P/libfsgpu_lrows.so $P/libfsgpu_lrowsds.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_lrows.log 2>&1 || { tail gpurun_out/r03/ab_lrows.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_lrows.log
