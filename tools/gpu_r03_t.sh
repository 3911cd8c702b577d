#!/bin/bash
# Round 3: batched backward passes — the GPU suite on the batch build, then an
# A/B of the round's head build, the batch code compiled out, and the batch build
# at several unwind_batch thresholds.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/pytest_gpu_batch.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu_batch.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_batch.log
PERF_AB_HASH=1 AB_TIMEOUT=300 timeout -k 10 800 bash tools/lib_ab.sh "$P/libfsgpu_head.so $P/libfsgpu_nobatch.so $P/libfsgpu_batch.so" c2,c3,c4 256 2 "default,unwind_batch=16,unwind_batch=48,unwind_batch=0" > gpurun_out/r03/ab_batch.log 2>&1 || { tail gpurun_out/r03/ab_batch.log; exit 1; }
cat gpurun_out/r03/ab_batch.log
