#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05at
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05at -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/r05at/bench_under_rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r05at/bench_under_rocprof.log; exit 1; }
st=$(find /tmp/r05at -name "*kernel_stats.csv" | head -1)
cp "$st" $GRAFT_REPO_ROOT/gpurun_out/r05at/bench_kernel_stats.csv
head -8 $GRAFT_REPO_ROOT/gpurun_out/r05at/bench_kernel_stats.csv | cut -c1-220
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r05at/bench_under_rocprof.log | cut -c1-300
