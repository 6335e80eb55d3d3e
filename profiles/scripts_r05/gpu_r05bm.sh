#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bm
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
export FLITE_LIB=f-lite_amd/tools/variants/tsplit/libflite_hip.so
for r in 1 2; do
  for s in 16 8 6 4 3 2 1; do
    FLITE_ATTN_TAIL_SPLIT=$s timeout -k 10 120 python -u f-lite_amd/tools/attn_halves_check.py time 2>&1 | grep time | sed "s/^/S<=$s /" | tee -a gpurun_out/r05bm/time.log || exit 1
  done
done
