#!/bin/bash
# Round 3: mesh-root cull variants (straight-line, error-bound margins, straight-line exact path, hoisted slopes); frame hashes across builds.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp PERF_AB_HASH=1
P=final-stage-path-tracer-2-0_amd
L="$P/libfsgpu.so $P/libfsgpu_bf.so $P/libfsgpu_bft.so $P/libfsgpu_bftl.so $P/libfsgpu_bfht.so $P/libfsgpu_bfhtl.so"
AB_TIMEOUT=200 timeout -k 10 1000 bash tools/lib_ab.sh "$L" c2,c3,c4 256 2 > gpurun_out/r03/ab_root_tol.log 2>&1 || { tail gpurun_out/r03/ab_root_tol.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_root_tol.log
