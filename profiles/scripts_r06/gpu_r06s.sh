#!/bin/bash
# round 6, call s: the bf16-residual GEMM epilogue with 16-B lanes (deal8 layout on load and store) -- its kernel
# tests, then 4 alternating image-level rounds against the 8-B-lane epilogue (FLITE_GEMM_RESID_NARROW=1)
set -o pipefail
mkdir -p gpurun_out/r06s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resid16.py > gpurun_out/r06s/resid16.log 2>&1 || { tail -30 gpurun_out/r06s/resid16.log; exit 1; }
tail -3 gpurun_out/r06s/resid16.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06s/bench_ab_resid_wide.log 4 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none" prod prod:FLITE_GEMM_RESID_NARROW=1 || { tail -20 gpurun_out/r06s/bench_ab_resid_wide.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06s/bench_ab_resid_wide.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
