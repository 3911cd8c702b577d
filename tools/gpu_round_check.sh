#!/bin/bash
# Round-end evidence on the GPU box (run from the repo root): the GPU test
# suite, smoke, the bench line and the rocprofv3 kernel-stats of the bench.
set -o pipefail
R=${1:-r03}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$R/pytest_gpu.log
bash tools/gpu_bench_prof.sh $R
