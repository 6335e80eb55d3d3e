#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 200 python -u f-lite_amd/tools/gemm_k_drift.py 2>&1 | grep -v amdgpu.ids || exit 1
done
