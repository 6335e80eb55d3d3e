#!/bin/bash
# round 6, call n: the reference's default 1344x896 pinned at CFG 6 (make_golden_full5.py's fp32 and bf16 CFG-6
# trajectories), and the CFG-1 cases again on the final build
set -o pipefail
mkdir -p gpurun_out/r06n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_depth.py -k "1344x896" -v -s --timeout 400 --timeout-method thread > gpurun_out/r06n/pytest_1344.log 2>&1 || { grep -E "dB|PASSED|SKIPPED|FAILED|Error" gpurun_out/r06n/pytest_1344.log | tail -20; exit 1; }
grep -E "dB|PASSED|SKIPPED|FAILED" gpurun_out/r06n/pytest_1344.log | tail -14
