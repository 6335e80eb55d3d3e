#!/bin/bash
# round 6, call q: the residual-storage decision re-measured on the final build: 4 alternating rounds at the metric
# workload (with the negative-prompt leg) and 2 at configs[4] (MXFP8, 1344x896, tiled VAE)
set -o pipefail
mkdir -p gpurun_out/r06q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06q/bench_ab_resid_1024.log 4 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 3 --probe none" prod prod:FLITE_RESID_BF16=0 || { tail -20 gpurun_out/r06q/bench_ab_resid_1024.log; exit 1; }
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06q/bench_ab_resid_fp8_1344.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none --fp8 --height 896 --width 1344 --vae-tiling" prod prod:FLITE_RESID_BF16=0 || { tail -20 gpurun_out/r06q/bench_ab_resid_fp8_1344.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r06q/bench_ab_resid_1024.log", "gpurun_out/r06q/bench_ab_resid_fp8_1344.log"):
    cur=None
    for l in open(f):
        if l.startswith("=="): cur=l.split()[1]
        elif l.startswith("{"):
            d=json.loads(l); print(f.split("/")[-1], cur, d["value"], d.get("value_with_negative_prompt"), d["config"]["residual_dtype"])
PY
