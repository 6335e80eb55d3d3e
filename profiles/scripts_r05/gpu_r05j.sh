#!/bin/bash
# round 5, call j: bench lines (1024^2 metric with the negative-prompt leg; 1344x896 bf16 and MXFP8 with the
# attention route policy) and the fp8 GEMM-class policies priced at 1344x896, 30 CFG-6 steps
set -o pipefail
mkdir -p gpurun_out/r05j
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_Q256_VERBOSE=1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05j/bench.log 2>&1 || { tail -5 gpurun_out/r05j/bench.log; exit 1; }
tail -1 gpurun_out/r05j/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1024', d['value'], d['value_with_negative_prompt'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --height 896 --width 1344 --vae-tiling --negative-images 0 > gpurun_out/r05j/bench_1344.log 2>&1 || { tail -5 gpurun_out/r05j/bench_1344.log; exit 1; }
tail -1 gpurun_out/r05j/bench_1344.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1344 bf16', d['value'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --height 896 --width 1344 --vae-tiling --fp8 --negative-images 0 > gpurun_out/r05j/bench_fp8.log 2>&1 || { tail -5 gpurun_out/r05j/bench_fp8.log; exit 1; }
tail -1 gpurun_out/r05j/bench_fp8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1344 fp8', d['value'], d['roofline']['frac'])"
FLITE_ATTN_Q256=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --height 896 --width 1344 --vae-tiling --fp8 --negative-images 0 > gpurun_out/r05j/bench_fp8_q128.log 2>&1 || { tail -5 gpurun_out/r05j/bench_fp8_q128.log; exit 1; }
tail -1 gpurun_out/r05j/bench_fp8_q128.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1344 fp8 (128-row attention)', d['value'])"
timeout -k 10 900 python -u f-lite_amd/tools/fp8_policy.py --images 2 --policies "none" --class-policies "gate_up;gate_up,down;down;qkv,proj,cross_q,cross_proj;gate_up,qkv" > gpurun_out/r05j/fp8_policy.log 2>&1 || { tail -5 gpurun_out/r05j/fp8_policy.log; exit 1; }
cat gpurun_out/r05j/fp8_policy.log | grep policy
