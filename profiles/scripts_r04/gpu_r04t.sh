#!/bin/bash
# round 4, call t: the default bench line (with the CPU baseline) on the final bench.py
set -o pipefail
mkdir -p gpurun_out/r04t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/r04t/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r04t/bench.log; exit 1; }
grep "^{" gpurun_out/r04t/bench.log > gpurun_out/r04t/bench_line.json
tail -1 gpurun_out/r04t/bench.log | cut -c1-300
