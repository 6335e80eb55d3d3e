#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05ag
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05ag/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --probe none --negative-images 0 --height 896 --width 1344 --vae-tiling --fp8 > $GRAFT_REPO_ROOT/gpurun_out/r05ag/trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r05ag/trace.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r05ag/trace.log | cut -c1-200
