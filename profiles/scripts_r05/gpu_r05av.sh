#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05av
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u f-lite_amd/tools/fp8_class_p3.py --policies "all@0;all@0,1;all@0,1,2,3;all@0,1,2,3,4,5,6,7;all@0,39;all@0,1,38,39;all@36,37,38,39;gate_up,qkv@0,1,2,3;down@0,1,2,3" > gpurun_out/r05av/fp8_block_p3.log 2>&1 || { tail -20 gpurun_out/r05av/fp8_block_p3.log; exit 1; }
grep '^{' gpurun_out/r05av/fp8_block_p3.log
timeout -k 10 600 python -u f-lite_amd/tools/fp8_policy.py --images 3 --policies "none;0;0,1;0,1,2,3;0,1,2,3,4,5,6,7" > gpurun_out/r05av/fp8_block_speed.log 2>&1 || { tail -20 gpurun_out/r05av/fp8_block_speed.log; exit 1; }
grep '^{' gpurun_out/r05av/fp8_block_speed.log
