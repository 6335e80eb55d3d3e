#!/bin/bash
# round 4, call a: new tests + default bench line
set -o pipefail
mkdir -p gpurun_out/r04a
export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/r04b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_gpu_dit.py::test_cfg_block0_dedup_matches_full_batch" \
  tests/test_gpu_apg_parallel.py \
  "tests/test_gpu_fp8.py::test_fp8_bf16_block_policy" \
  "tests/test_gpu_fp8.py::test_fp8_256_free_running_30_steps" \
  tests/test_gpu_weights_update.py "tests/test_gpu_full_depth.py::test_10b_1024_30_steps_vs_reference" > gpurun_out/r04a/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/r04a/pytest.log; exit 1; }
grep -E "dB|passed|failed" gpurun_out/r04a/pytest.log | tail -30
timeout -k 10 600 python -u bench.py > gpurun_out/r04a/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r04a/bench.log; exit 1; }
tail -1 gpurun_out/r04a/bench.log
FLITE_LIB=f-lite_amd/tools/variants/stamps/libflite_hip.so timeout -k 10 300 python -u f-lite_amd/tools/attn_stamps.py run > gpurun_out/r04a/stamps.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/r04a/stamps.log; exit 1; }
cat gpurun_out/r04a/stamps.log
