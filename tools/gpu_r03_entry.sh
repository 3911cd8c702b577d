set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "every_option" > gpurun_out/r03/opt_parity.log 2>&1 || { tail -20 gpurun_out/r03/opt_parity.log; exit 1; }
tail -2 gpurun_out/r03/opt_parity.log
timeout -k 10 400 python -u tools/perf_ab.py "default,park_entry=24,park_entry=32,park_entry=40,park_entry=48" c4 256 2 > gpurun_out/r03/ab_entry_c4.log 2>&1 || exit 1
cat gpurun_out/r03/ab_entry_c4.log
timeout -k 10 400 python -u tools/perf_ab.py "default,park_entry_small=16,park_entry_small=24,park_entry_small=32" c3 256 2 > gpurun_out/r03/ab_entry_c3.log 2>&1 || exit 1
cat gpurun_out/r03/ab_entry_c3.log
