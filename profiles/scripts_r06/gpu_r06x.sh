#!/bin/bash
# round 6, call x: the whole GPU suite on the final round-6 tree (16-B-lane residual epilogues, SK_FAN switch), then smoke
set -o pipefail
mkdir -p gpurun_out/r06x
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/r06x/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r06x/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06x/smoke.log 2>&1 || { tail -5 gpurun_out/r06x/smoke.log; exit 1; }
tail -2 gpurun_out/r06x/smoke.log
