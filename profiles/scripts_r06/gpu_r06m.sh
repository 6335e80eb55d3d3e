#!/bin/bash
# round 6, call m: the 7B MXFP8 CFG-6 policy test, and the world-size-8 rehearsal (7B replicas) on the final build
set -o pipefail
mkdir -p gpurun_out/r06m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_depth.py -k "fp8_7b_cfg6" -v -s --timeout 240 --timeout-method thread > gpurun_out/r06m/pytest_fp8_7b_cfg6.log 2>&1 || { tail -30 gpurun_out/r06m/pytest_fp8_7b_cfg6.log; exit 1; }
grep -E "dB|PASSED|FAILED" gpurun_out/r06m/pytest_fp8_7b_cfg6.log | tail -3
FLITE_BENCH_REHEARSAL=1 timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29563 bench.py --gpus 8 --model 7b --steps 1 --warmup 1 --negative-images 1 --no-cpu-baseline > gpurun_out/r06m/rehearsal_gpus8.log 2>&1 || { tail -20 gpurun_out/r06m/rehearsal_gpus8.log; exit 1; }
tail -1 gpurun_out/r06m/rehearsal_gpus8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal', d['n_gpus'], d['value'], d['value_with_negative_prompt'], d['distributed']['process_group'], d['config']['residual_dtype'])"
