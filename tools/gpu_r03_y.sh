#!/bin/bash
# Round 3: wave priority of the shading block / backward pass, -O2, no jump tables and the
# scheduler's metric bias, against the product build; frames must be identical.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
P=final-stage-path-tracer-2-0_amd
L=""
for v in "" _sp1 _up1 _sup1 _o2 _nojt _bias0; do L="$L $P/libfsgpu$v.so"; done
PERF_AB_HASH=1 AB_TIMEOUT=300 timeout -k 10 1000 bash tools/lib_ab.sh "$L" c2,c3,c4 256 2 > gpurun_out/r03/ab_prio.log 2>&1 || { tail gpurun_out/r03/ab_prio.log; exit 1; }
grep -E "==|variant|md5" gpurun_out/r03/ab_prio.log
