#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05au
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u f-lite_amd/tools/fp8_class_p3.py --policies "none;all;gate_up,qkv;gate_up,down;gate_up;qkv,proj,cross_q,cross_proj;down;all@0,1,2,3" > gpurun_out/r05au/fp8_class_p3.log 2>&1 || { tail -20 gpurun_out/r05au/fp8_class_p3.log; exit 1; }
grep '^{' gpurun_out/r05au/fp8_class_p3.log
