#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bb
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
A="--warmup 1 --no-cpu-baseline --negative-images 0"
for v in "1 3" "2 2" "4 1" "1 3" "2 2" "4 1"; do
  set -- $v
  timeout -k 10 300 python -u bench.py $A --images-per-gpu $1 --steps $2 > gpurun_out/r05bb/bench_b$1.log 2>&1 || { tail -20 gpurun_out/r05bb/bench_b$1.log; exit 1; }
  python3 -c "import json; l=[x for x in open('gpurun_out/r05bb/bench_b$1.log') if x.startswith('{\"metric')][-1]; d=json.loads(l); print('images_per_gpu', $1, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d.get('mfma_util_image'))" | tee -a gpurun_out/r05bb/summary.txt
done
