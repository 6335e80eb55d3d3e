#!/bin/bash
# round 6, call k: the existing A/B switches re-checked on the bf16-residual build (their defaults were tuned with
# the fp32 stream): weight read-aheads off, the norm2 read-ahead off, 224-row tiles off; two alternating rounds
set -o pipefail
mkdir -p gpurun_out/r06k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06k/bench_ab_switches.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none" prod prod:FLITE_NO_WPREFETCH=1 prod:FLITE_NO_NORM_PF=1 prod:FLITE_GEMM_NO_BM224=1 || { tail -20 gpurun_out/r06k/bench_ab_switches.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06k/bench_ab_switches.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
