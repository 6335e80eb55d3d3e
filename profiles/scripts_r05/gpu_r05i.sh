#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_Q256_VERBOSE=1
timeout -k 10 400 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,self1344,self512,self1536,cross --rounds 2 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "attention" --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
