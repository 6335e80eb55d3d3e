#!/bin/bash
# round 5, call c: 256-row attention after the P-operand fix: diagnostic over plans, ops tests, DiT/fp8 tests, bench
set -o pipefail
mkdir -p gpurun_out/r05c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for plan in default "384,1" "0,10"; do
  echo "== plan $plan"
  if [ "$plan" = default ]; then
    timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py > gpurun_out/r05c/diag_default.log 2>&1 || exit 1
    tail -3 gpurun_out/r05c/diag_default.log | cut -c1-400
  else
    FLITE_Q256_PLAN="$plan" timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | tail -3 | cut -c1-400 || exit 1
  fi
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v -k "attention" --timeout 120 --timeout-method thread -s > gpurun_out/r05c/pytest_ops.log 2>&1 || { echo "ops failed"; grep -E "FAILED|Error|error|q256" gpurun_out/r05c/pytest_ops.log | head -30; exit 1; }
grep -E "q256|passed|failed" gpurun_out/r05c/pytest_ops.log | tail -12
timeout -k 10 900 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_fp8.py -m gpu -x -q -rs --timeout 300 --timeout-method thread -s > gpurun_out/r05c/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r05c/pytest.log | head -20; tail -30 gpurun_out/r05c/pytest.log; exit 1; }
tail -3 gpurun_out/r05c/pytest.log
grep -E "fp8 classes|collapse" gpurun_out/r05c/pytest.log | head -20
timeout -k 10 400 python -u bench.py --no-cpu-baseline --probe attn > gpurun_out/r05c/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r05c/bench.log; exit 1; }
tail -1 gpurun_out/r05c/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['negative_prompt'], d['distributed']['process_group'], d['distributed']['context_broadcast_ms'], d['roofline'])"
timeout -k 10 300 python -u f-lite_amd/tools/q256_bench.py > gpurun_out/r05c/q256_bench.log 2>&1 || exit 1
cat gpurun_out/r05c/q256_bench.log
FLITE_Q256_MIN_KEYS=256 timeout -k 10 300 python -u f-lite_amd/tools/q256_bench.py --rounds 2 2>&1 | grep cross
