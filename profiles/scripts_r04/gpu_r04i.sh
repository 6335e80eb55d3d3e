#!/bin/bash
# round 4, call i: uniform-context collapse in the MXFP8 path -- equivalence test, fp8 suite, fp8 policy table,
# fp8 bench A/B (configs[4] 1344x896)
set -o pipefail
mkdir -p gpurun_out/r04i
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s \
  "tests/test_gpu_dit.py::test_uniform_context_collapse_matches_full_computation" \
  "tests/test_gpu_dit.py::test_cfg_block0_dedup_matches_full_batch" \
  tests/test_gpu_fp8.py 2>&1 | tee gpurun_out/r04i/pytest.log | grep -E "dB|passed|failed|FAILED|Error" || { echo "pytest failed"; tail -30 gpurun_out/r04i/pytest.log; exit 1; }
timeout -k 10 600 python -u f-lite_amd/tools/fp8_policy.py --images 2 > gpurun_out/r04i/fp8_policy.log 2>&1 || { echo "fp8 policy failed"; tail -20 gpurun_out/r04i/fp8_policy.log; exit 1; }
cat gpurun_out/r04i/fp8_policy.log | cut -c1-300
for arm in on off on; do
  if [ $arm = off ]; then export FLITE_NO_CTX_COLLAPSE=1; else unset FLITE_NO_CTX_COLLAPSE; fi
  timeout -k 10 400 python -u bench.py --fp8 --height 896 --width 1344 --vae-tiling --no-cpu-baseline 2>&1 | tee -a gpurun_out/r04i/bench_fp8_$arm.log | grep "^{" | cut -c1-200 || { echo "bench failed"; exit 1; }
done
