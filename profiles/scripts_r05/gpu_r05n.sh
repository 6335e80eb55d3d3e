#!/bin/bash
# round 5, call n: V^T fragments of phase B read at the tail of phase A (128- and 256-row kernels): parity + timing A/B
set -o pipefail
mkdir -p gpurun_out/r05n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:|q128:" | cut -c1-200 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or attn" > gpurun_out/r05n/pytest_attn.log 2>&1 || { tail -30 gpurun_out/r05n/pytest_attn.log; exit 1; }
tail -1 gpurun_out/r05n/pytest_attn.log
for r in 1 2; do
for v in product base128 base256; do
  echo "== $v"
  if [ $v = product ]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$v/libflite_hip.so; fi
  FLITE_LIB=$lib timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,self1344,cross --rounds 2 2>&1 | grep -E "q256|q128" || exit 1
done
done
