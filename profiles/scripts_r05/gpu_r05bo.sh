#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bo
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B=FLITE_LIB=$GRAFT_REPO_ROOT/f-lite_amd/tools/variants/fused/libflite_hip.so
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py $B --preset 10b --depth 4 --size 256 > gpurun_out/r05bo/eq_10b.log 2>&1 || { tail -20 gpurun_out/r05bo/eq_10b.log; exit 1; }
tail -3 gpurun_out/r05bo/eq_10b.log
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py $B --preset 7b --depth 12 --size 256 > gpurun_out/r05bo/eq_7b.log 2>&1 || { tail -20 gpurun_out/r05bo/eq_7b.log; exit 1; }
tail -3 gpurun_out/r05bo/eq_7b.log
FLITE_LIB=$GRAFT_REPO_ROOT/f-lite_amd/tools/variants/fused/libflite_hip.so timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bo/pytest_dit.log 2>&1 || { tail -30 gpurun_out/r05bo/pytest_dit.log; exit 1; }
tail -1 gpurun_out/r05bo/pytest_dit.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r05bo/bench_ab_norm3_bc.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0" prod fused || { tail -20 gpurun_out/r05bo/bench_ab_norm3_bc.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r05bo/bench_ab_norm3_bc.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
