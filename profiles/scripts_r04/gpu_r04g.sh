#!/bin/bash
# round 4, call g: uniform-context collapse -- equivalence tests, parity at the metric config, bench A/B
set -o pipefail
mkdir -p gpurun_out/r04g
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s \
  "tests/test_gpu_dit.py::test_uniform_context_collapse_matches_full_computation" \
  "tests/test_gpu_dit.py::test_cfg_block0_dedup_matches_full_batch" \
  "tests/test_gpu_dit.py::test_sampling_loop_vs_oracle" \
  "tests/test_gpu_full_depth.py::test_10b_1024_forward" \
  "tests/test_gpu_full_depth.py::test_1024_free_running_4_steps" \
  "tests/test_gpu_full_depth.py::test_256_free_running_30_steps" \
  "tests/test_gpu_full_depth.py::test_10b_1024_30_steps_vs_reference" \
  "tests/test_gpu_cfg_parallel.py" 2>&1 | tee gpurun_out/r04g/pytest.log | grep -E "dB|passed|failed|FAILED|Error" || { echo "pytest failed"; tail -30 gpurun_out/r04g/pytest.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee gpurun_out/r04g/bench_collapse.log | grep "^{" | cut -c1-300 || { echo "bench failed"; exit 1; }
FLITE_NO_CTX_COLLAPSE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee gpurun_out/r04g/bench_nocollapse.log | grep "^{" | cut -c1-300 || { echo "bench failed"; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee gpurun_out/r04g/bench_collapse2.log | grep "^{" | cut -c1-300 || { echo "bench failed"; exit 1; }
