#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ah
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
  for v in model always; do
    if [ $v = always ]; then export FLITE_FP8_SK_ALWAYS=1; else unset FLITE_FP8_SK_ALWAYS; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --negative-images 0 --height 896 --width 1344 --vae-tiling --fp8 > gpurun_out/r05ah/bench_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r05ah/bench_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/r05ah/bench_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'])"
  done
done
