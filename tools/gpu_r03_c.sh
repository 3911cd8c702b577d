#!/bin/bash
# Round 3, call 3: GPU suite, radiance-row layout / NOWALK kernel A/B, write traffic.
set -o pipefail
mkdir -p gpurun_out/r03/writes2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_c.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu_c.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu_c.log
timeout -k 10 200 python -u tools/perf_ab.py "default,lds_rows=0" c2 256 3 > gpurun_out/r03/ab_nowalk.log 2>&1 || { tail gpurun_out/r03/ab_nowalk.log; exit 1; }
cat gpurun_out/r03/ab_nowalk.log
P=final-stage-path-tracer-2-0_amd
AB_TIMEOUT=200 timeout -k 10 600 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_nw7.so $P/libfsgpu_nw8.so" c2 256 2 > gpurun_out/r03/ab_nowalk_waves.log 2>&1 || { tail gpurun_out/r03/ab_nowalk_waves.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_nowalk_waves.log
AB_TIMEOUT=200 timeout -k 10 700 bash tools/lib_ab.sh "$P/libfsgpu_radplanar.so $P/libfsgpu.so $P/libfsgpu_radnt.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_rad.log 2>&1 || { tail gpurun_out/r03/ab_rad.log; exit 1; }
grep -E "==|variant" gpurun_out/r03/ab_rad.log
for sc in c4 c2; do
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03/writes2/$sc -o pmc -- python3 bench.py --scene $sc --steps 1 --warmup 0 --spp 512 --no-cpu > gpurun_out/r03/writes2/$sc.out 2>&1 || { echo "writes $sc failed"; tail -5 gpurun_out/r03/writes2/$sc.out; exit 1; }
done
echo writes done
