#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05af
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2 3; do
  for v in off on; do
    if [ $v = on ]; then export FLITE_DOWN_PF=1; else unset FLITE_DOWN_PF; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --negative-images 0 > gpurun_out/r05af/bench_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r05af/bench_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/r05af/bench_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'])"
  done
done
