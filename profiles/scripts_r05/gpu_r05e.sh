#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in product noholds; do
  if [ "$v" = product ]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$v/libflite_hip.so; fi
  echo "== $v"
  FLITE_LIB=$lib timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py > gpurun_out/r05e/diag_$v.log 2>&1 || { tail gpurun_out/r05e/diag_$v.log; exit 1; }
  grep -E "row 33|row 97|q256:|q128:" gpurun_out/r05e/diag_$v.log | cut -c1-400
  FLITE_LIB=$lib FLITE_Q256_PLAN="384,10" timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:" | cut -c1-300
done
