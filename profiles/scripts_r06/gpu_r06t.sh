#!/bin/bash
# round 6, call t: the MXFP8 bf16-residual epilogue with 16-B lanes -- its kernel tests (bit-equal to the fp32-stream
# epilogue rounded once), the fp8 suite, then alternating image-level rounds against the 8-B-lane epilogue
# (FLITE_GEMM_RESID_NARROW=1) at configs[4] (MXFP8, 1344x896, tiled VAE) and at the 1024^2 metric size
set -o pipefail
mkdir -p gpurun_out/r06t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resid16.py tests/test_gpu_fp8.py > gpurun_out/r06t/fp8.log 2>&1 || { tail -30 gpurun_out/r06t/fp8.log; exit 1; }
tail -3 gpurun_out/r06t/fp8.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06t/bench_ab_resid_wide_fp8_1344.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none --fp8 --height 896 --width 1344 --vae-tiling" prod prod:FLITE_GEMM_RESID_NARROW=1 || { tail -20 gpurun_out/r06t/bench_ab_resid_wide_fp8_1344.log; exit 1; }
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06t/bench_ab_resid_wide_fp8_1024.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none --fp8" prod prod:FLITE_GEMM_RESID_NARROW=1 || { tail -20 gpurun_out/r06t/bench_ab_resid_wide_fp8_1024.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r06t/bench_ab_resid_wide_fp8_1344.log", "gpurun_out/r06t/bench_ab_resid_wide_fp8_1024.log"):
    cur=None
    for l in open(f):
        if l.startswith("=="): cur=l.split()[1]
        elif l.startswith("{"):
            d=json.loads(l); print(f.split("/")[-1], cur, d["value"], d["ms_per_step"])
PY
