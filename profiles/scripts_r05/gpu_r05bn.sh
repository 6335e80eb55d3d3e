#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bn
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_final -o run -- python3 -u bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --negative-images 0 > gpurun_out/r05bn/bench.log 2>&1 || { tail -20 gpurun_out/r05bn/bench.log; exit 1; }
csv=$(find /tmp/prof_final -name "*kernel_trace.csv" | head -1)
st=$(find /tmp/prof_final -name "*kernel_stats.csv" | head -1)
cp "$st" gpurun_out/r05bn/nograph_kernel_stats.csv
python3 f-lite_amd/tools/trace_by_grid.py "$csv" attn gemm_bf16 rmsnorm > gpurun_out/r05bn/grid.txt
head -14 gpurun_out/r05bn/grid.txt
