#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05be
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10 200"
FLITE_ATTN_HALVES=0 $T python -u f-lite_amd/tools/attn_halves_check.py check /tmp/h0.pt > gpurun_out/r05be/check_h0.log 2>&1 || { tail -20 gpurun_out/r05be/check_h0.log; exit 1; }
FLITE_ATTN_HALVES=100000 $T python -u f-lite_amd/tools/attn_halves_check.py check /tmp/hall.pt > gpurun_out/r05be/check_hall.log 2>&1 || { tail -20 gpurun_out/r05be/check_hall.log; exit 1; }
FLITE_ATTN_HALVES=5 $T python -u f-lite_amd/tools/attn_halves_check.py check /tmp/h5.pt > gpurun_out/r05be/check_h5.log 2>&1 || { tail -20 gpurun_out/r05be/check_h5.log; exit 1; }
$T python -u f-lite_amd/tools/attn_halves_check.py check /tmp/hplan.pt > gpurun_out/r05be/check_plan.log 2>&1 || { tail -20 gpurun_out/r05be/check_plan.log; exit 1; }
grep -h worst gpurun_out/r05be/check_*.log
$T python -u f-lite_amd/tools/attn_halves_check.py compare /tmp/h0.pt /tmp/hall.pt > gpurun_out/r05be/compare_h0_hall.log 2>&1 || exit 1
$T python -u f-lite_amd/tools/attn_halves_check.py compare /tmp/h0.pt /tmp/hplan.pt > gpurun_out/r05be/compare_h0_plan.log 2>&1 || exit 1
cat gpurun_out/r05be/compare_h0_hall.log
for n in plan 0 32 64 96 128 160 192 256 plan 0; do
  if [ $n = plan ]; then unset FLITE_ATTN_HALVES; else export FLITE_ATTN_HALVES=$n; fi
  $T python -u f-lite_amd/tools/attn_halves_check.py time $( [ $n = plan ] && echo --self ) 2>&1 | grep time | tee -a gpurun_out/r05be/time.log || exit 1
done
