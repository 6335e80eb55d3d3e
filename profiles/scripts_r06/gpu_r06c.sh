#!/bin/bash
# round 6, call c: the bf16-residual tests (tests/test_gpu_resid16.py), the per-block MXFP8 class policies against
# the reference at 1024^2 CFG 1, and the speed of the candidates at 1024^2
set -o pipefail
mkdir -p gpurun_out/r06c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_resid16.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06c/pytest_resid16.log 2>&1 || { tail -40 gpurun_out/r06c/pytest_resid16.log; exit 1; }
tail -1 gpurun_out/r06c/pytest_resid16.log
timeout -k 10 900 python -u f-lite_amd/tools/fp8_block_policy.py > gpurun_out/r06c/fp8_block_policy.log 2>&1 || { tail -20 gpurun_out/r06c/fp8_block_policy.log; exit 1; }
cat gpurun_out/r06c/fp8_block_policy.log | grep '^{'
