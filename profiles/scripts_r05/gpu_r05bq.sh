#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bq
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/f-lite_amd/tools/variants/fp8fold/libflite_hip.so
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py FLITE_LIB=$V --preset 10b --depth 4 --size 256 --fp8 > gpurun_out/r05bq/eq_10b_fp8.log 2>&1 || { tail -20 gpurun_out/r05bq/eq_10b_fp8.log; exit 1; }
tail -2 gpurun_out/r05bq/eq_10b_fp8.log
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py FLITE_LIB=$V --preset 10b --depth 4 --size 256 > gpurun_out/r05bq/eq_10b.log 2>&1 || { tail -20 gpurun_out/r05bq/eq_10b.log; exit 1; }
tail -2 gpurun_out/r05bq/eq_10b.log
FLITE_LIB=$V timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bq/pytest.log 2>&1 || { tail -30 gpurun_out/r05bq/pytest.log; exit 1; }
tail -1 gpurun_out/r05bq/pytest.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r05bq/bench_ab_fp8fold.log 2 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0 --fp8 --height 896 --width 1344 --vae-tiling" prod fp8fold || { tail -20 gpurun_out/r05bq/bench_ab_fp8fold.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r05bq/bench_ab_fp8fold.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
