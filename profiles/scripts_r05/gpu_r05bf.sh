#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bf
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py -m gpu -x -v -s --timeout 250 --timeout-method thread -k "num_images or sampling_loop" > gpurun_out/r05bf/pytest.log 2>&1 || { tail -30 gpurun_out/r05bf/pytest.log; exit 1; }
grep -E "PASS|FAIL|dB" gpurun_out/r05bf/pytest.log | cut -c1-200; tail -1 gpurun_out/r05bf/pytest.log
