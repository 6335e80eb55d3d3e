#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ad
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1100 python -u bench.py --steps 1 --warmup 1 --negative-images 0 --cpu-baseline-full 2 > gpurun_out/r05ad/bench_cpu_full.log 2>&1 || { tail -20 gpurun_out/r05ad/bench_cpu_full.log; exit 1; }
tail -1 gpurun_out/r05ad/bench_cpu_full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['cpu_baseline'])[:900])"
