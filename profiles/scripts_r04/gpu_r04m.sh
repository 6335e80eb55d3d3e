#!/bin/bash
# round 4, call m: metric-config parity with the reference bf16 floor and the uint8 images
set -o pipefail
mkdir -p gpurun_out/r04m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s -rs \
  "tests/test_gpu_full_depth.py::test_10b_1024_30_steps_vs_reference" 2>&1 | tee gpurun_out/r04m/pytest.log | grep -E "dB|passed|failed|FAILED|Error|SKIP" || { echo "pytest failed"; tail -30 gpurun_out/r04m/pytest.log; exit 1; }
