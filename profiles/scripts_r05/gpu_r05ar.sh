#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ar
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in m32 m16 m32 m16; do
  if [ $v = m16 ]; then export FLITE_ATTN_M16=1; else unset FLITE_ATTN_M16; fi
  echo "== $v"
  timeout -k 10 200 python -u f-lite_amd/tools/attn_m16_check.py --loop-like > gpurun_out/r05ar/loop_like_$v.log 2>&1 || { tail -20 gpurun_out/r05ar/loop_like_$v.log; exit 1; }
  grep time gpurun_out/r05ar/loop_like_$v.log | tail -4
done
