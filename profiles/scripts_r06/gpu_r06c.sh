#!/bin/bash
# round 6, call c: the bf16-residual tests (tests/test_gpu_resid16.py, both storage types explicitly), the default
# bench line with the bf16 residual default, and the per-block MXFP8 class policies against the reference at 1024^2
# CFG 1
set -o pipefail
mkdir -p gpurun_out/r06c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_resid16.py tests/test_gpu_full_depth.py -k "resid or 7b_256_free" -v -s --timeout 300 --timeout-method thread > gpurun_out/r06c/pytest_resid16.log 2>&1 || { tail -40 gpurun_out/r06c/pytest_resid16.log; exit 1; }
tail -1 gpurun_out/r06c/pytest_resid16.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r06c/bench.log 2>&1 || { tail -5 gpurun_out/r06c/bench.log; exit 1; }
tail -1 gpurun_out/r06c/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1024', d['value'], d['value_with_negative_prompt'], d['roofline']['frac'], d['config']['residual_dtype'])"
timeout -k 10 900 python -u f-lite_amd/tools/fp8_block_policy.py > gpurun_out/r06c/fp8_block_policy.log 2>&1 || { tail -20 gpurun_out/r06c/fp8_block_policy.log; exit 1; }
grep '^{' gpurun_out/r06c/fp8_block_policy.log
