#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bl
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r05bl/bench_ab_livechunks.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0" prod prev || { tail -20 gpurun_out/r05bl/bench_ab_livechunks.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r05bl/bench_ab_livechunks.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
