#!/bin/bash
# Round 3, call 6: the POOL schedule (parity, then A/B against PARKED), the 7-wave parked kernel.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "pool or every_option or zoo" > gpurun_out/r03/pytest_pool.log 2>&1 || { tail -40 gpurun_out/r03/pytest_pool.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r03/pytest_pool.log | tail -12
timeout -k 10 600 python -u tools/perf_ab.py "schedule=parked,schedule=pool,schedule=pool@pool_refill=32,schedule=pool@pool_refill=48,schedule=pool@pool_sync=0" c4,c3 256 2 > gpurun_out/r03/ab_pool.log 2>&1 || { tail gpurun_out/r03/ab_pool.log; exit 1; }
cat gpurun_out/r03/ab_pool.log
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_s7.so" c3,c4 256 2 > gpurun_out/r03/ab_susp7.log 2>&1 || { tail gpurun_out/r03/ab_susp7.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_susp7.log
AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_poolhbm.so" c3,c4 256 2 schedule=pool > gpurun_out/r03/ab_pool_rows.log 2>&1 || { tail gpurun_out/r03/ab_pool_rows.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_pool_rows.log
