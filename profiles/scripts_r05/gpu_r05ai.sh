#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
echo "== q128 / auto"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes self --rounds 2 2>&1 | grep -E "q128|q256" || exit 1
for plan in "0,1" "0,4" "0,10" "0,16" "64,10" "128,4" "128,10" "128,16" "192,10" "256,10" "384,10" "384,1"; do
  echo "== plan $plan"; FLITE_Q256_PLAN="$plan" timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes self --rounds 2 2>&1 | grep -E "q256:" || exit 1
done
