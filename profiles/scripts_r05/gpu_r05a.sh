#!/bin/bash
# round 5, call a: the 256-row attention kernel (ops test), the set_context / fp8 collapse fixes,
# then the bench line with the negative-prompt leg
set -o pipefail
mkdir -p gpurun_out/r05a
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v -k "attention" --timeout 120 --timeout-method thread -s > gpurun_out/r05a/pytest_ops.log 2>&1 || { echo "ops failed"; grep -E "FAILED|Error|error|q256" gpurun_out/r05a/pytest_ops.log | head -30; tail -30 gpurun_out/r05a/pytest_ops.log; exit 1; }
grep -E "q256|passed|failed" gpurun_out/r05a/pytest_ops.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_fp8.py -m gpu -x -q -rs --timeout 300 --timeout-method thread -s > gpurun_out/r05a/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r05a/pytest.log | head -20; tail -30 gpurun_out/r05a/pytest.log; exit 1; }
tail -3 gpurun_out/r05a/pytest.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05a/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r05a/bench.log; exit 1; }
tail -1 gpurun_out/r05a/bench.log | cut -c1-300
tail -1 gpurun_out/r05a/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['negative_prompt'], d['distributed'], d['roofline'])"
