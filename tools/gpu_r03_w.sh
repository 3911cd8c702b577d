#!/bin/bash
# Round 3: the 32-B quantized BVH nodes — GPU suite on it, then an A/B against the head build.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/pytest_gpu_qnodes.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu_qnodes.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_qnodes.log
PERF_AB_HASH=1 AB_TIMEOUT=300 timeout -k 10 800 bash tools/lib_ab.sh "$P/libfsgpu_head.so $P/libfsgpu_q.so" c2,c3,c4 256 3 > gpurun_out/r03/ab_qnodes.log 2>&1 || { tail gpurun_out/r03/ab_qnodes.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_qnodes.log
