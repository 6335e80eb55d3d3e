#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ab
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl_single_rank.py -m gpu -x -v -s --timeout 250 --timeout-method thread > gpurun_out/r05ab/pytest.log 2>&1 || { tail -40 gpurun_out/r05ab/pytest.log; exit 1; }
grep -E "PASS|FAIL|process group|rel " gpurun_out/r05ab/pytest.log | cut -c1-250; tail -1 gpurun_out/r05ab/pytest.log
