#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05aq
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in m32 m16; do
  if [ $v = m16 ]; then export FLITE_ATTN_M16=1; else unset FLITE_ATTN_M16; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_$v -o run -- python3 -u bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --negative-images 0 > gpurun_out/r05aq/bench_$v.log 2>&1 || { tail -20 gpurun_out/r05aq/bench_$v.log; exit 1; }
  csv=$(find /tmp/prof_$v -name "*kernel_trace.csv" | head -1)
  python3 f-lite_amd/tools/trace_by_grid.py "$csv" attn gemm_bf16 rmsnorm > gpurun_out/r05aq/grid_$v.txt
  echo "== $v"; head -14 gpurun_out/r05aq/grid_$v.txt
done
