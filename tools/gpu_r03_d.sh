#!/bin/bash
# Round 3, call 4: GPU suite on the branch-free object loop, then its A/B.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_d.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu_d.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_d.log
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 800 bash tools/lib_ab.sh "$P/libfsgpu_bf0.so $P/libfsgpu.so $P/libfsgpu_rootslopes.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_branchfree.log 2>&1 || { tail gpurun_out/r03/ab_branchfree.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_branchfree.log
