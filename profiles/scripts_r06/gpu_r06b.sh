#!/bin/bash
# round 6, call b: the bf16 residual stream: a same-box image A/B at 1024^2 against the fp32
# residual (same library, env switch), then the whole GPU suite with FLITE_RESID_BF16=1
set -o pipefail
mkdir -p gpurun_out/r06b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06b/bench_ab_resid16.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0" prod prod:FLITE_RESID_BF16=1 || { tail -20 gpurun_out/r06b/bench_ab_resid16.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06b/bench_ab_resid16.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"], d["config"]["residual_dtype"])
PY
FLITE_RESID_BF16=1 timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/r06b/pytest_resid16.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r06b/pytest_resid16.log | tail -15
exit $rc
