#!/bin/bash
# round 5, call d: hazard hypotheses for the 256-row attention (variant libraries via FLITE_LIB)
set -o pipefail
mkdir -p gpurun_out/r05d
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in q256same q256samen; do
  echo "== $v"
  if [ "$v" = product ]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$v/libflite_hip.so; fi
  FLITE_LIB=$lib timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py > gpurun_out/r05d/diag_$v.log 2>&1 || exit 1
  tail -4 gpurun_out/r05d/diag_$v.log | cut -c1-300
done
