#!/bin/bash
# round 4, call r: norm2's cross-q weight read-ahead under the collapse (norm2 now covers the cond rows only): A/B
set -o pipefail
mkdir -p gpurun_out/r04r
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for arm in pf nopf pf nopf; do
  if [ $arm = nopf ]; then export FLITE_NO_NORM_PF=1; else unset FLITE_NO_NORM_PF; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee -a gpurun_out/r04r/bench_$arm.log | grep "^{" | cut -c1-160 || { echo "bench failed"; exit 1; }
done
