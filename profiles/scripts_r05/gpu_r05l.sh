#!/bin/bash
# round 5, call l: 256-row attention cycle anatomy under ablations (diagnostic builds: outputs not valid), and the
# configs[1] 30-step test with its PSNR printout
set -o pipefail
mkdir -p gpurun_out/r05l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in q256stamps st_nodma st_nokread st_kahead4 st_nosmx st_novread; do
  echo "== $v"
  FLITE_LIB=f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run > gpurun_out/r05l/stamps_$v.log 2>&1 || { tail -5 gpurun_out/r05l/stamps_$v.log; exit 1; }
  grep "self 2x4112 H12 whole" gpurun_out/r05l/stamps_$v.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_depth.py -m gpu -x -v -s --timeout 500 --timeout-method thread -k "30_steps_vs_reference and 7b" > gpurun_out/r05l/pytest_7b_1024_30.log 2>&1 || { tail -30 gpurun_out/r05l/pytest_7b_1024_30.log; exit 1; }
grep -E "dB|passed|failed" gpurun_out/r05l/pytest_7b_1024_30.log | cut -c1-250
