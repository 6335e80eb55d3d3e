#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for plan in "128,10" "384,1" "0,1"; do
  echo "== plan $plan"
  FLITE_Q256_PLAN="$plan" FLITE_LIB=f-lite_amd/tools/variants/q256stamps/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run 2>&1 | grep -A6 "self 2x4112 H12: realtime" || exit 1
done
