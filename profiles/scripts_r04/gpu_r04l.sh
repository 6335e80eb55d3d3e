#!/bin/bash
# round 4, call l: round evidence on the collapse build (smoke, bench line, kernel trace, gate/up counter passes)
set -o pipefail
mkdir -p gpurun_out/r04l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/round_evidence.sh gpurun_out/r04l || { echo "evidence failed"; tail -20 gpurun_out/r04l/*.log; exit 1; }
tail -2 gpurun_out/r04l/smoke.log
tail -1 gpurun_out/r04l/bench.log | cut -c1-400
python f-lite_amd/tools/trace_split.py $(find gpurun_out/r04l/trace -name "*kernel_trace.csv") > gpurun_out/r04l/trace_split.txt 2>&1; cat gpurun_out/r04l/trace_split.txt
cp $(find gpurun_out/r04l/trace -name "*kernel_stats.csv") gpurun_out/r04l/nograph_kernel_stats.csv
cp $(find gpurun_out/r04l/gemm_time -name "*kernel_stats.csv") gpurun_out/r04l/gemm_kernel_stats.csv
python f-lite_amd/tools/pmc_traffic.py gpurun_out/r04l/pmc_fetch gpurun_out/r04l/pmc_write gpurun_out/r04l/pmc_mfma gpurun_out/r04l/pmc_traffic.json > gpurun_out/r04l/pmc_reduce.log 2>&1; cat gpurun_out/r04l/pmc_reduce.log | head -30
rm -rf gpurun_out/r04l/trace
