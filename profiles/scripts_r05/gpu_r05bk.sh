#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bk
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bk/pytest.log 2>&1 || { tail -30 gpurun_out/r05bk/pytest.log; exit 1; }
tail -1 gpurun_out/r05bk/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05bk/smoke.log 2>&1 || { tail -20 gpurun_out/r05bk/smoke.log; exit 1; }
tail -2 gpurun_out/r05bk/smoke.log
timeout -k 10 330 python -u bench.py > gpurun_out/r05bk/bench.log 2>&1 || { tail -20 gpurun_out/r05bk/bench.log; exit 1; }
tail -1 gpurun_out/r05bk/bench.log | cut -c1-600
