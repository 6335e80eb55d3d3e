#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 200 python -u f-lite_amd/tools/down_round_fit.py 2>&1 | grep -v amdgpu.ids || exit 1
FLITE_GEMM_NO_SK=1 timeout -k 10 200 python -u f-lite_amd/tools/down_round_fit.py 2>&1 | grep -v amdgpu.ids | sed 's/^/no_sk /' || exit 1
done
