#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05aw
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "first_blocks or free_running" > gpurun_out/r05aw/pytest.log 2>&1 || { tail -30 gpurun_out/r05aw/pytest.log; exit 1; }
grep -E "PASS|FAIL|dB" gpurun_out/r05aw/pytest.log | cut -c1-200; tail -1 gpurun_out/r05aw/pytest.log
