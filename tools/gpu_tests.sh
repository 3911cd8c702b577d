#!/bin/bash
# GPU test suite on the box (run from the repo root): pytest -m gpu with a
# per-test limit; the log and the parity records land in gpurun_out/$R.
set -o pipefail
R=${1:-r02}
shift
mkdir -p gpurun_out/$R
rm -f gpurun_out/parity_records.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "$@" > gpurun_out/$R/pytest_gpu.log 2>&1
rc=$?
[ -f gpurun_out/parity_records.jsonl ] && mv gpurun_out/parity_records.jsonl gpurun_out/$R/
tail -5 gpurun_out/$R/pytest_gpu.log
exit $rc
