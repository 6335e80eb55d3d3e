#!/bin/bash
# round 4, call c: fp8 precision policies (configs[4]) + latency-mode rehearsal lines (not measurements)
set -o pipefail
mkdir -p gpurun_out/r04c
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u f-lite_amd/tools/fp8_policy.py --images 2 > gpurun_out/r04c/fp8_policy.log 2>&1 || { echo "fp8 policy failed"; tail -20 gpurun_out/r04c/fp8_policy.log; exit 1; }
cat gpurun_out/r04c/fp8_policy.log
for m in cfg-parallel sp sp-ring; do
  FLITE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --mode $m --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04c/rehearsal_$m.log 2>&1 || { echo "rehearsal $m failed"; tail -20 gpurun_out/r04c/rehearsal_$m.log; exit 1; }
  tail -1 gpurun_out/r04c/rehearsal_$m.log
done
