#!/bin/bash
# Prints VGPRs / scratch / occupancy of every kernel in fs_device.hip
cd /root/repo/final-stage-path-tracer-2-0_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -Icsrc -c ${1:-csrc/fs_device.hip} -o /tmp/vg.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed 's/.*remark: *//; s/ \[-Rpass.*//' \
 | paste - - - - | sed 's/Function Name: _ZN2fs3dev//' | awk -F'\t' '{printf "%-60s %s | %s | %s\n", substr($1,1,60), $2, $3, $4}'
