#!/bin/bash
# round 6, call j: the 16-B-lane bf16 norm, one row per 128-thread workgroup: op + fp8 + residual tests, a same-box image A/B
# against the one-row kernel (FLITE_NORM_ROW1=1), and norm kernel times from a --no-graph trace
set -o pipefail
mkdir -p gpurun_out/r06j
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py tests/test_gpu_resid16.py tests/test_gpu_dit.py -q --timeout 300 --timeout-method thread -rA > gpurun_out/r06j/pytest.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error" gpurun_out/r06j/pytest.log | tail -20; exit 1; }
tail -1 gpurun_out/r06j/pytest.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06j/bench_ab_h16.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0" prod prod:FLITE_NORM_ROW1=1 || { tail -20 gpurun_out/r06j/bench_ab_h16.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06j/bench_ab_h16.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06j/trace -o run -- python3 bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none > gpurun_out/r06j/trace.log 2>&1 || { tail -5 gpurun_out/r06j/trace.log; exit 1; }
grep -i "rmsnorm" gpurun_out/r06j/trace/run_kernel_stats.csv | cut -c1-170
