#!/bin/bash
# round 6, call a: the default bench line with the whole-step CPU baseline, then the
# world-size-8 bench path rehearsed end to end on one card with 7B replicas
set -o pipefail
mkdir -p gpurun_out/r06a
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r06a/bench.log 2>&1 || { tail -20 gpurun_out/r06a/bench.log; exit 1; }
tail -1 gpurun_out/r06a/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cpu_baseline']; print('1024', d['value'], d['value_with_negative_prompt'], d['roofline']['frac'], c['value'], c['sample'], c['components_check']['ratio_to_value'])"
FLITE_BENCH_REHEARSAL=1 timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --model 7b --steps 1 --warmup 1 --negative-images 1 --no-cpu-baseline > gpurun_out/r06a/rehearsal_gpus8.log 2>&1 || { tail -20 gpurun_out/r06a/rehearsal_gpus8.log; exit 1; }
tail -1 gpurun_out/r06a/rehearsal_gpus8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal', d['n_gpus'], d['value'], d['distributed']['process_group'], d['distributed']['backend'])"
