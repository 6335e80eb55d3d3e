#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05as
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FLITE_ATTN_M16=2 timeout -k 10 200 python -u f-lite_amd/tools/attn_m16_check.py --no-time > gpurun_out/r05as/check_v64.log 2>&1 || { tail -20 gpurun_out/r05as/check_v64.log; exit 1; }
grep -E "worst" gpurun_out/r05as/check_v64.log
for v in 0 1 2 0 1 2; do
  echo "== FLITE_ATTN_M16=$v"
  FLITE_ATTN_M16=$v timeout -k 10 200 python -u f-lite_amd/tools/attn_m16_check.py --loop-like > gpurun_out/r05as/loop_like_$v.log 2>&1 || { tail -20 gpurun_out/r05as/loop_like_$v.log; exit 1; }
  grep time gpurun_out/r05as/loop_like_$v.log | tail -4
done
