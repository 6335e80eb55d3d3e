#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ao
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 python -u f-lite_amd/tools/attn_m16_check.py > gpurun_out/r05ao/check_m32.log 2>&1 || { tail -20 gpurun_out/r05ao/check_m32.log; exit 1; }
FLITE_ATTN_M16=1 timeout -k 10 240 python -u f-lite_amd/tools/attn_m16_check.py > gpurun_out/r05ao/check_m16.log 2>&1 || { tail -20 gpurun_out/r05ao/check_m16.log; exit 1; }
timeout -k 10 120 python -u f-lite_amd/tools/attn_m16_check.py --time-only > gpurun_out/r05ao/time_m32b.log 2>&1 || { tail -20 gpurun_out/r05ao/time_m32b.log; exit 1; }
FLITE_ATTN_M16=1 timeout -k 10 120 python -u f-lite_amd/tools/attn_m16_check.py --time-only > gpurun_out/r05ao/time_m16b.log 2>&1 || { tail -20 gpurun_out/r05ao/time_m16b.log; exit 1; }
for f in check_m32 check_m16 time_m32b time_m16b; do echo "== $f"; grep -E "kernel|worst|time|DIFF|nan|finite False" gpurun_out/r05ao/$f.log; done
