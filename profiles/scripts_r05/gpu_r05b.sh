#!/bin/bash
# round 5, call b: locate the 256-row attention kernel's wrong segment (plans forced per process)
set -o pipefail
mkdir -p gpurun_out/r05b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for plan in default "0,1" "384,1" "0,10" "128,4"; do
  echo "== plan $plan"
  if [ "$plan" = default ]; then
    timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | tail -4 || exit 1
  else
    FLITE_Q256_PLAN="$plan" timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | tail -4 || exit 1
  fi
done
