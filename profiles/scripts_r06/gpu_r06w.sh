#!/bin/bash
# round 6, call w: stream-K forced on every short GEMM launch with a partial last round (qkv 4.64 rounds, proj and
# cross-q 1.55 rounds at 256-row tiles), FLITE_GEMM_SK_FAN=2/3, against the model's choice (qkv, proj: data-parallel)
set -o pipefail
mkdir -p gpurun_out/r06w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FLITE_GEMM_SK_FAN=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_resid16.py::test_10b_1024_30_steps_bf16_residual_vs_reference" -s > gpurun_out/r06w/parity_fan2.log 2>&1 || { tail -20 gpurun_out/r06w/parity_fan2.log; exit 1; }
grep "dB" gpurun_out/r06w/parity_fan2.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06w/bench_ab_sk_fan.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none" prod prod:FLITE_GEMM_SK_FAN=2 prod:FLITE_GEMM_SK_FAN=3 || { tail -20 gpurun_out/r06w/bench_ab_sk_fan.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06w/bench_ab_sk_fan.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
