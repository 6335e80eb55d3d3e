#!/bin/bash
# round 4, call b: attention schedule variants (A/B alternating, fp32-checked) + bit-identity + stamps
set -o pipefail
export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/r04b
VARIANTS_CHECK=1 timeout -k 10 900 python -u f-lite_amd/tools/variants.py run attention base rs ql qlld qsld qlqsld qlqsldvb qlqsldvb2 --rounds 2 > gpurun_out/r04b/variants.log 2>&1 || { echo "variants failed"; tail -30 gpurun_out/r04b/variants.log; exit 1; }
tail -10 gpurun_out/r04b/variants.log
for v in base ql qlld qlqsld; do
  FLITE_LIB=f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r04b/eq_$v.pt > gpurun_out/r04b/eq_$v.log 2>&1 || { echo "dump $v failed"; tail gpurun_out/r04b/eq_$v.log; exit 1; }
done
for v in ql qlld qlqsld; do echo "== base vs $v"; python f-lite_amd/tools/attn_equal.py compare gpurun_out/r04b/eq_base.pt gpurun_out/r04b/eq_$v.pt | tail -10; done
rm -f gpurun_out/r04b/*.pt
FLITE_LIB=f-lite_amd/tools/variants/stamps_qlqsld/libflite_hip.so timeout -k 10 300 python -u f-lite_amd/tools/attn_stamps.py run > gpurun_out/r04b/stamps_qlqsld.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/r04b/stamps_qlqsld.log; exit 1; }
cat gpurun_out/r04b/stamps_qlqsld.log
