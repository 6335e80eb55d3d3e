#!/bin/bash
# round 5, call s: down projection data parallel on 224-row tiles (FLITE_GEMM_NO_SK) vs stream-K over 256-row tiles
set -o pipefail
mkdir -p gpurun_out/r05s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="import sys; sys.path.insert(0,'f-lite_amd/tools'); import variants; r=variants.time_gemms(); print({k:(round(v[0]*1e3,1), round(v[1]/2516.6,3), v[2]) for k,v in r.items()})"
for r in 1 2; do
  echo "== sk";   VARIANTS_CHECK=1 timeout -k 10 200 python -u -c "$T" 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== no_sk"; FLITE_GEMM_NO_SK=1 VARIANTS_CHECK=1 timeout -k 10 200 python -u -c "$T" 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
  for v in sk no_sk; do
    if [ $v = no_sk ]; then export FLITE_GEMM_NO_SK=1; else unset FLITE_GEMM_NO_SK; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --negative-images 0 > gpurun_out/r05s/bench_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r05s/bench_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/r05s/bench_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'])"
  done
done
