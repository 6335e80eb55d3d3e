#!/bin/bash
# round 4, call j: full GPU suite on the collapse build (bf16 + MXFP8)
set -o pipefail
mkdir -p gpurun_out/r04j
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -s > gpurun_out/r04j/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r04j/pytest.log | head -20; tail -30 gpurun_out/r04j/pytest.log; exit 1; }
tail -5 gpurun_out/r04j/pytest.log
