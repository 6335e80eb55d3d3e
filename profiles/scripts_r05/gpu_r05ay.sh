#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ay
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
A="--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0"
for r in 1 2; do
  for v in bf16 fp8all fp8b8; do
    case $v in bf16) X="";; fp8all) X="--fp8";; fp8b8) X="--fp8 --fp8-bf16-blocks 0,1,2,3,4,5,6,7";; esac
    timeout -k 10 240 python -u bench.py $A $X > gpurun_out/r05ay/bench_${v}_$r.log 2>&1 || { tail -20 gpurun_out/r05ay/bench_${v}_$r.log; exit 1; }
    python3 -c "import json,sys; l=[x for x in open('gpurun_out/r05ay/bench_${v}_$r.log') if x.startswith('{\"metric')][-1]; d=json.loads(l); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
