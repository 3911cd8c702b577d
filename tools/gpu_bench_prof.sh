#!/bin/bash
# Round profiling script (runs on the GPU box from the repo root): smoke, the
# bench line (C4, with the CPU baseline), the other configs' lines, and the
# rocprofv3 kernel-trace stats of the C4 bench command.
set -o pipefail
R=${1:-r03}
mkdir -p gpurun_out/$R
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/$R/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench failed; tail -20 gpurun_out/$R/bench.err; exit 1; }
cat gpurun_out/$R/bench.json
for sc in c2 c3; do
  timeout -k 10 300 python bench.py --scene $sc --no-cpu > gpurun_out/$R/bench_$sc.json 2> gpurun_out/$R/bench_$sc.err || { echo bench $sc failed; tail -20 gpurun_out/$R/bench_$sc.err; exit 1; }
  cut -c1-200 gpurun_out/$R/bench_$sc.json
done
timeout -k 10 300 python bench.py --width 3840 --height 2160 --steps 2 --no-cpu > gpurun_out/$R/bench_c5frame.json 2> gpurun_out/$R/bench_c5frame.err || { echo bench c5 failed; tail -20 gpurun_out/$R/bench_c5frame.err; exit 1; }
cut -c1-200 gpurun_out/$R/bench_c5frame.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/$R/prof_bench.json 2> gpurun_out/$R/prof.err || { echo rocprof failed; tail -20 gpurun_out/$R/prof.err; exit 1; }
find gpurun_out/$R/prof -name "*stats*" | head
