#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ax
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_full_depth.py -m gpu -x -v -s --timeout 400 --timeout-method thread -k "fp8_first_blocks" > gpurun_out/r05ax/pytest.log 2>&1 || { tail -30 gpurun_out/r05ax/pytest.log; exit 1; }
grep -E "PASS|FAIL|dB" gpurun_out/r05ax/pytest.log | cut -c1-220; tail -1 gpurun_out/r05ax/pytest.log
