#!/bin/bash
# round 4, call d: full GPU suite on the new attention (q pre-scale, unshifted exp2, delayed row sum, cheap
# descriptors) + the round evidence (smoke, bench line, kernel trace, gate/up counter passes)
set -o pipefail
mkdir -p gpurun_out/r04d
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -s > gpurun_out/r04d/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r04d/pytest.log | head -20; tail -30 gpurun_out/r04d/pytest.log; exit 1; }
tail -3 gpurun_out/r04d/pytest.log
bash f-lite_amd/tools/round_evidence.sh gpurun_out/r04d || { echo "evidence failed"; exit 1; }
tail -1 gpurun_out/r04d/bench.log
python f-lite_amd/tools/trace_split.py $(find gpurun_out/r04d/trace -name "*kernel_trace.csv") > gpurun_out/r04d/trace_split.txt 2>&1; cat gpurun_out/r04d/trace_split.txt
head -12 $(find gpurun_out/r04d/trace -name "*kernel_stats.csv") | cut -c1-160
