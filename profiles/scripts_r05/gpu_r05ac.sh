#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ac
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FLITE_BENCH_PG=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --negative-images 0 > gpurun_out/r05ac/bench_pg1.log 2>&1 || { tail -20 gpurun_out/r05ac/bench_pg1.log; exit 1; }
tail -1 gpurun_out/r05ac/bench_pg1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['distributed']))"
