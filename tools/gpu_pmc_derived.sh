#!/bin/bash
# rocprofv3 derived metrics (one per pass) on the bench workload; a metric the
# tool does not know on this GPU is reported and skipped.
# usage: tools/gpu_pmc_derived.sh ROUND SPP WIDTH HEIGHT METRIC...
set -o pipefail
R=$1; SPP=$2; W=$3; H=$4; shift 4
OUT=gpurun_out/$R/derived_${W}x${H}
mkdir -p $OUT
export TMPDIR=/tmp
for m in "$@"; do
  timeout -s KILL 150 rocprofv3 --pmc $m --output-format csv -d $OUT/$m -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --spp $SPP --no-cpu --width $W --height $H > $OUT/$m.out 2> $OUT/$m.err
  rc=$?
  echo "$m rc=$rc"
  [ $rc -eq 137 ] && { echo "$m killed at its limit: stopping"; exit 1; }
done
exit 0
