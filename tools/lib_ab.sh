#!/bin/bash
# A/B of builds of libfsgpu.so on one box: alternating processes.
# usage: tools/lib_ab.sh "libA libB ..." scenes spp rounds [fs_options variant, default: the defaults]
LIBS=$1; SC=${2:-c2,c3,c4}; SPP=${3:-32}; R=${4:-2}; MODE=${5:-default}
for i in $(seq 1 $R); do
  for L in $LIBS; do
    echo "== $L"
    FSAMD_GPU_LIB=$PWD/$L timeout -k 10 ${AB_TIMEOUT:-150} python tools/perf_ab.py $MODE $SC $SPP 1 || exit 1
  done
done
