#!/bin/bash
# round 4, call u: final full GPU suite (incl. the 7B 1024^2 CFG-6 fixture) + smoke
set -o pipefail
mkdir -p gpurun_out/r04u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -s > gpurun_out/r04u/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r04u/pytest.log | head -20; tail -30 gpurun_out/r04u/pytest.log; exit 1; }
tail -4 gpurun_out/r04u/pytest.log
grep -E "1024\^2 30-step|uint8 image" gpurun_out/r04u/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04u/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r04u/smoke.log; exit 1; }
tail -1 gpurun_out/r04u/smoke.log
