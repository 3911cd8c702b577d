#!/bin/bash
# Round 3: device-compiler scheduling strategies and traversal wave priority 0 / 3 (same source, -mllvm flags on the device
# compile only) against the product build; frames must be identical.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
PERF_AB_HASH=1 AB_TIMEOUT=300 timeout -k 10 900 bash tools/lib_ab.sh "$P/libfsgpu.so $P/libfsgpu_ilp.so $P/libfsgpu_clause.so $P/libfsgpu_trk.so $P/libfsgpu_prio0.so $P/libfsgpu_prio3.so" c2,c3,c4 256 2 > gpurun_out/r03/ab_sched.log 2>&1 || { tail gpurun_out/r03/ab_sched.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_sched.log
