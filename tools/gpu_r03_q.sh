#!/bin/bash
# Round 3: GPU suite on the lane-major-rows build.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_lrows.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r03/pytest_gpu_lrows.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_lrows.log
