#!/bin/bash
# round 6, call d: the reference's default 1344x896 pinned at CFG 1 (make_golden_full5.py's first trajectory), the
# configs[2] / configs[4] bench lines with the bf16 residual default (bf16, all-MXFP8, and the quality policy
# blocks 0-7 bf16, at 1344x896 and 1024^2), and a --no-graph kernel trace of the metric workload
set -o pipefail
mkdir -p gpurun_out/r06d
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_depth.py -k "1344x896" -v -s --timeout 400 --timeout-method thread > gpurun_out/r06d/pytest_1344.log 2>&1 || { tail -40 gpurun_out/r06d/pytest_1344.log; exit 1; }
grep -E "dB|PASSED|SKIPPED|FAILED" gpurun_out/r06d/pytest_1344.log | tail -12
run() {  # name, args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --negative-images 0 $2 > gpurun_out/r06d/bench_$1.log 2>&1 || { tail -5 gpurun_out/r06d/bench_$1.log; exit 1; }
  tail -1 gpurun_out/r06d/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'], d['config']['residual_dtype'])"
}
run 1344_bf16 "--height 896 --width 1344 --vae-tiling"
run 1344_fp8 "--height 896 --width 1344 --vae-tiling --fp8"
run 1344_fp8_b07 "--height 896 --width 1344 --vae-tiling --fp8 --fp8-bf16-blocks 0,1,2,3,4,5,6,7"
run 1024_fp8 "--fp8"
run 1024_fp8_b07 "--fp8 --fp8-bf16-blocks 0,1,2,3,4,5,6,7"
run 7b_1024 "--model 7b"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d/trace -o run -- python3 bench.py --no-graph --steps 1 --warmup 1 --no-cpu-baseline --negative-images 0 --probe none > gpurun_out/r06d/trace.log 2>&1 || { tail -5 gpurun_out/r06d/trace.log; exit 1; }
f=$(ls gpurun_out/r06d/trace/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r06d/nograph_kernel_stats.csv && head -14 gpurun_out/r06d/nograph_kernel_stats.csv | cut -c1-150
