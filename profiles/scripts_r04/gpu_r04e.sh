#!/bin/bash
# round 4, call e: attention pack-delay variants + stamps; fp8 precision policies (configs[4]); latency-mode rehearsal
set -o pipefail
mkdir -p gpurun_out/r04e
export PYTHONUNBUFFERED=1
VARIANTS_CHECK=1 timeout -k 10 600 python -u f-lite_amd/tools/variants.py run attention base prod pd pdvb --rounds 3 > gpurun_out/r04e/variants.log 2>&1 || { echo "variants failed"; tail -30 gpurun_out/r04e/variants.log; exit 1; }
tail -6 gpurun_out/r04e/variants.log
for v in prod pd; do
  FLITE_LIB=f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r04e/eq_$v.pt > gpurun_out/r04e/eq_$v.log 2>&1 || { echo "dump $v failed"; exit 1; }
done
python f-lite_amd/tools/attn_equal.py compare gpurun_out/r04e/eq_prod.pt gpurun_out/r04e/eq_pd.pt | tail -10; rm -f gpurun_out/r04e/*.pt
FLITE_LIB=f-lite_amd/tools/variants/stamps_pd/libflite_hip.so timeout -k 10 300 python -u f-lite_amd/tools/attn_stamps.py run > gpurun_out/r04e/stamps_pd.log 2>&1 || { echo "stamps failed"; exit 1; }
cat gpurun_out/r04e/stamps_pd.log
timeout -k 10 600 python -u f-lite_amd/tools/fp8_policy.py --images 2 > gpurun_out/r04e/fp8_policy.log 2>&1 || { echo "fp8 policy failed"; tail -20 gpurun_out/r04e/fp8_policy.log; exit 1; }
cat gpurun_out/r04e/fp8_policy.log
for m in cfg-parallel sp sp-ring; do
  FLITE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --mode $m --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04e/rehearsal_$m.log 2>&1 || { echo "rehearsal $m failed"; tail -20 gpurun_out/r04e/rehearsal_$m.log; exit 1; }
  grep "^{" gpurun_out/r04e/rehearsal_$m.log | tail -1 | cut -c1-400
done
