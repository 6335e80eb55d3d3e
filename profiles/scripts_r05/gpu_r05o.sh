#!/bin/bash
# round 5, call o: 256-row attention built without SLP vectorisation (no v_pk_add_f32 row sums in the PV phase)
set -o pipefail
mkdir -p gpurun_out/r05o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:|q128:" | cut -c1-200 || exit 1
FLITE_LIB=f-lite_amd/tools/variants/q256stamps/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run > gpurun_out/r05o/stamps.log 2>&1 || { tail -5 gpurun_out/r05o/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05o/stamps.log
for r in 1 2; do
for v in product base256; do
  echo "== $v"
  if [ $v = product ]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$v/libflite_hip.so; fi
  FLITE_LIB=$lib timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,self1344 --rounds 2 2>&1 | grep -E "q256" || exit 1
done
done
