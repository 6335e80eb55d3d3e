#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05am
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FLITE_BENCH_REHEARSAL=1 timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 1 --warmup 1 --negative-images 1 --no-cpu-baseline > gpurun_out/r05am/rehearsal_gpus8.log 2>&1 || { tail -20 gpurun_out/r05am/rehearsal_gpus8.log; exit 1; }
tail -1 gpurun_out/r05am/rehearsal_gpus8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('value_with_negative_prompt'), d['n_gpus'], json.dumps(d['distributed']['process_group']), d['distributed']['context_broadcast_ms'])"
