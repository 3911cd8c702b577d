#!/bin/bash
# Round 3, call 2: GPU suite, root-cull A/B, undistorted phase split, write-stream breakdown.
set -o pipefail
mkdir -p gpurun_out/r03/writes
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu.log
AB_TIMEOUT=200 timeout -k 10 700 bash tools/lib_ab.sh "final-stage-path-tracer-2-0_amd/libfsgpu_rootold.so final-stage-path-tracer-2-0_amd/libfsgpu.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_root_pairs.log 2>&1 || { tail gpurun_out/r03/ab_root_pairs.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_root_pairs.log
timeout -k 10 300 python -u tools/phase_prof.py c4,c2,c3 64 > gpurun_out/r03/phase.log 2>&1 || { tail gpurun_out/r03/phase.log; exit 1; }
cat gpurun_out/r03/phase.log
for v in "" _meas_NO_LVL _meas_NO_RAD; do
  FSAMD_GPU_LIB=$PWD/final-stage-path-tracer-2-0_amd/libfsgpu$v.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03/writes/w$v -o pmc -- python3 bench.py --steps 1 --warmup 0 --spp 512 --no-cpu > gpurun_out/r03/writes/w$v.out 2>&1 || { echo "writes $v failed"; tail -5 gpurun_out/r03/writes/w$v.out; exit 1; }
done
echo writes done
