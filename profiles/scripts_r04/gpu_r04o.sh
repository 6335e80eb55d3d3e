#!/bin/bash
# round 4, call o: the collapsed rows' update on a side stream (FLITE_CTX_OVERLAP): bit-equality, bench A/B
set -o pipefail
mkdir -p gpurun_out/r04o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u f-lite_amd/tools/env_equal.py FLITE_CTX_OVERLAP=1 2>&1 | tee gpurun_out/r04o/equal.log || { echo "equal failed"; exit 1; }
for arm in on off on off; do
  if [ $arm = on ]; then export FLITE_CTX_OVERLAP=1; else unset FLITE_CTX_OVERLAP; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee -a gpurun_out/r04o/bench_$arm.log | grep "^{" | cut -c1-160 || { echo "bench failed"; exit 1; }
done
