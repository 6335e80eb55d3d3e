#!/bin/bash
# round 5, call p: 128-row attention reads P in place in the PV MFMAs (no NOP-form copies): bit equality + timing A/B
set -o pipefail
mkdir -p gpurun_out/r05p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_ATTN_Q256=0
FLITE_LIB=f-lite_amd/f_lite/libflite_hip.so timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r05p/new.pt > gpurun_out/r05p/eq.log 2>&1 || { tail -5 gpurun_out/r05p/eq.log; exit 1; }
FLITE_LIB=f-lite_amd/tools/variants/base128/libflite_hip.so timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r05p/old.pt >> gpurun_out/r05p/eq.log 2>&1 || { tail -5 gpurun_out/r05p/eq.log; exit 1; }
timeout -k 10 60 python -u f-lite_amd/tools/attn_equal.py compare gpurun_out/r05p/new.pt gpurun_out/r05p/old.pt 2>&1 | tail -4 || exit 1
rm -f gpurun_out/r05p/*.pt
for r in 1 2 3; do
for v in product base128; do
  echo "== $v"
  if [ $v = product ]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$v/libflite_hip.so; fi
  FLITE_LIB=$lib timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
done
done
