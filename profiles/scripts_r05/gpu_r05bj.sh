#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bj
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10 200"
$T python -u f-lite_amd/tools/attn_equal.py dump /tmp/base.pt > gpurun_out/r05bj/eq.log 2>&1 || exit 1
FLITE_LIB=f-lite_amd/tools/variants/live/libflite_hip.so $T python -u f-lite_amd/tools/attn_equal.py dump /tmp/new.pt >> gpurun_out/r05bj/eq.log 2>&1 || exit 1
$T python -u f-lite_amd/tools/attn_equal.py compare /tmp/base.pt /tmp/new.pt >> gpurun_out/r05bj/eq.log 2>&1; echo "compare rc $?"
grep -E "identical|DIFFERENT" gpurun_out/r05bj/eq.log
for r in 1 2 3; do
  $T python -u f-lite_amd/tools/attn_halves_check.py time 2>&1 | grep time | sed 's/^/base /' | tee -a gpurun_out/r05bj/time.log || exit 1
  FLITE_LIB=f-lite_amd/tools/variants/live/libflite_hip.so $T python -u f-lite_amd/tools/attn_halves_check.py time 2>&1 | grep time | sed "s/^/new  /" | tee -a gpurun_out/r05bj/time.log || exit 1
done
