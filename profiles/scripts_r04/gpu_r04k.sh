#!/bin/bash
# round 4, call k: GEMM static wave priority A/B (guide T5 static form), GEMM shapes then image
set -o pipefail
mkdir -p gpurun_out/r04k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd f-lite_amd
timeout -k 10 600 python -u tools/variants.py run gemm g_base g_prio_young g_prio_old --rounds 3 2>&1 | tee ../gpurun_out/r04k/variants.log | tail -30 || { echo "variants failed"; exit 1; }
cd ..
for v in g_base g_prio_young g_base g_prio_young; do
  FLITE_LIB=$PWD/f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee -a gpurun_out/r04k/bench_$v.log | grep "^{" | cut -c1-160 || { echo "bench failed"; exit 1; }
done
