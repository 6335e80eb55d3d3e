#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05z
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py tests/test_gpu_dit.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attention or attn or dit or collapse" > gpurun_out/r05z/pytest.log 2>&1 || { tail -30 gpurun_out/r05z/pytest.log; exit 1; }
tail -2 gpurun_out/r05z/pytest.log
