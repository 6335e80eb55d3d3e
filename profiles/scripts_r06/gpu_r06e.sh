#!/bin/bash
# round 6, call e: the two-rows-per-workgroup bf16 norm kernel: op tests, bit-identity against the one-row kernel
# (FLITE_NORM_ROW1=1) in the bf16 and MXFP8 loops, a same-box image A/B, and a --no-graph kernel trace
set -o pipefail
mkdir -p gpurun_out/r06e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "rmsnorm" -q --timeout 120 --timeout-method thread > gpurun_out/r06e/pytest_norm.log 2>&1 || { tail -30 gpurun_out/r06e/pytest_norm.log; exit 1; }
tail -1 gpurun_out/r06e/pytest_norm.log
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py FLITE_NORM_ROW1=1 --preset 10b --depth 4 --size 256 > gpurun_out/r06e/eq_bf16.log 2>&1 || { tail -20 gpurun_out/r06e/eq_bf16.log; exit 1; }
cat gpurun_out/r06e/eq_bf16.log
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py FLITE_NORM_ROW1=1 --preset 10b --depth 4 --size 256 --fp8 > gpurun_out/r06e/eq_fp8.log 2>&1 || { tail -20 gpurun_out/r06e/eq_fp8.log; exit 1; }
cat gpurun_out/r06e/eq_fp8.log
bash f-lite_amd/tools/bench_ab.sh gpurun_out/r06e/bench_ab_norm2.log 3 "--steps 3 --warmup 1 --no-cpu-baseline --negative-images 0" prod prod:FLITE_NORM_ROW1=1 || { tail -20 gpurun_out/r06e/bench_ab_norm2.log; exit 1; }
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06e/bench_ab_norm2.log"):
    if l.startswith("=="): cur=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(cur, d["value"], d["ms_per_step"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e/trace -o run -- python3 bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none > gpurun_out/r06e/trace.log 2>&1 || { tail -5 gpurun_out/r06e/trace.log; exit 1; }
grep -i "rmsnorm" gpurun_out/r06e/trace/run_kernel_stats.csv | cut -c1-170
