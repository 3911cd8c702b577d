#!/bin/bash
# Round 3: GPU suite on the straight-line mesh-root cull build, then its A/B (frame hashes across builds).
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_root.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r03/pytest_gpu_root.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_root.log
P=final-stage-path-tracer-2-0_amd
PERF_AB_HASH=1 AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu_base.so $P/libfsgpu_bfhtl.so $P/libfsgpu.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_root_lite.log 2>&1 || { tail gpurun_out/r03/ab_root_lite.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_root_lite.log
