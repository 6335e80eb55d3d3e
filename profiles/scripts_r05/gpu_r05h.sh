#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in qreg2 qreg3; do
  lib=f-lite_amd/tools/variants/$v/libflite_hip.so
  echo "== $v"
  FLITE_LIB=$lib timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:|q128:" | cut -c1-200 || exit 1
  FLITE_LIB=$lib timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,self1344 --rounds 2 2>&1 | grep -E "q256|q128" || exit 1
done
