#!/bin/bash
# round 6, call u: the whole GPU suite on the build with 16-B-lane residual / SwiGLU-bf16 epilogues, smoke, then the
# default bench line (the driver's N=1 command) and configs[4]
set -o pipefail
mkdir -p gpurun_out/r06u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/r06u/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r06u/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06u/smoke.log 2>&1 || { tail -5 gpurun_out/r06u/smoke.log; exit 1; }
tail -2 gpurun_out/r06u/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06u/bench_default.log 2>&1 || { tail -20 gpurun_out/r06u/bench_default.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --negative-images 0 --fp8 --height 896 --width 1344 --vae-tiling > gpurun_out/r06u/bench_fp8_1344.log 2>&1 || { tail -20 gpurun_out/r06u/bench_fp8_1344.log; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_default", "bench_fp8_1344"):
    for l in open(f"gpurun_out/r06u/{f}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d.get("value_with_negative_prompt"), (d.get("roofline") or {}).get("frac"), (d.get("cpu_baseline") or {}).get("value"))
PY
