#!/bin/bash
# round 6, call p: stream-K switches re-checked on the bf16 residual (the down GEMM's finisher epilogue changed), and
# the 1344x896 attention route (256-row kernel by prediction vs forced off)
set -o pipefail
mkdir -p gpurun_out/r06p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06p/bench_ab_sk.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none" prod prod:FLITE_GEMM_NO_STREAM_K=1 prod:FLITE_GEMM_NO_SK=1 || { tail -20 gpurun_out/r06p/bench_ab_sk.log; exit 1; }
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06p/bench_ab_q256_1344.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none --height 896 --width 1344 --vae-tiling" prod prod:FLITE_ATTN_Q256=0 || { tail -20 gpurun_out/r06p/bench_ab_q256_1344.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r06p/bench_ab_sk.log", "gpurun_out/r06p/bench_ab_q256_1344.log"):
    cur=None
    for l in open(f):
        if l.startswith("=="): cur=l.split()[1]
        elif l.startswith("{"):
            d=json.loads(l); print(f.split("/")[-1], cur, d["value"], d["ms_per_step"])
PY
