#!/bin/bash
# round 4, call f: split-phase attention variants (+ stamps); SP / SP-ring rehearsal lines (2 steps, not measurements)
set -o pipefail
mkdir -p gpurun_out/r04f
export PYTHONUNBUFFERED=1
VARIANTS_CHECK=1 timeout -k 10 600 python -u f-lite_amd/tools/variants.py run attention base prod spl splf --rounds 3 2>&1 | tee gpurun_out/r04f/variants.log | grep -E "^round|median|^base|^prod|^spl" || { echo "variants failed"; exit 1; }
for v in prod spl splf; do
  FLITE_LIB=f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r04f/eq_$v.pt > gpurun_out/r04f/eq_$v.log 2>&1 || { echo "dump $v failed"; exit 1; }
done
python f-lite_amd/tools/attn_equal.py compare gpurun_out/r04f/eq_prod.pt gpurun_out/r04f/eq_spl.pt | tail -10
python f-lite_amd/tools/attn_equal.py compare gpurun_out/r04f/eq_prod.pt gpurun_out/r04f/eq_splf.pt | tail -10; rm -f gpurun_out/r04f/*.pt
FLITE_LIB=f-lite_amd/tools/variants/stamps_spl/libflite_hip.so timeout -k 10 300 python -u f-lite_amd/tools/attn_stamps.py run 2>&1 | tee gpurun_out/r04f/stamps_spl.log || { echo "stamps failed"; exit 1; }
for m in sp sp-ring; do
  FLITE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --mode $m --steps 1 --warmup 0 --sample-steps 2 --no-cpu-baseline 2>&1 | tee gpurun_out/r04f/rehearsal_$m.log | grep -E "^\{|Error|error" | cut -c1-600 || { echo "rehearsal $m failed"; exit 1; }
done
