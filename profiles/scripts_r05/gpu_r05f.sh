#!/bin/bash
# round 5, call f: where the 256-row kernel's time goes: plans, an exact one-round shape
set -o pipefail
mkdir -p gpurun_out/r05f
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_Q256_VERBOSE=1
timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self --rounds 2 2>&1 | grep -v amdgpu.ids || exit 1
for plan in "0,1" "0,4" "128,1" "128,8" "192,8" "384,8"; do
  echo "== plan $plan"
  FLITE_Q256_PLAN="$plan" timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes self --rounds 2 2>&1 | grep -E "q256|\[q256\]" || exit 1
done
