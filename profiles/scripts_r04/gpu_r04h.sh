#!/bin/bash
# round 4, call h: kernel trace of the collapse build (per-kernel split of the sampling loop)
set -o pipefail
mkdir -p gpurun_out/r04h
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h/trace -o run -- python3 bench.py --no-graph --steps 1 \
  --warmup 1 --no-cpu-baseline --probe none > gpurun_out/r04h/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/r04h/trace.log; exit 1; }
python f-lite_amd/tools/trace_split.py $(find gpurun_out/r04h/trace -name "*kernel_trace.csv") > gpurun_out/r04h/trace_split.txt 2>&1; cat gpurun_out/r04h/trace_split.txt
cp $(find gpurun_out/r04h/trace -name "*kernel_stats.csv") gpurun_out/r04h/nograph_kernel_stats.csv
head -14 gpurun_out/r04h/nograph_kernel_stats.csv | cut -c1-160
rm -rf gpurun_out/r04h/trace
