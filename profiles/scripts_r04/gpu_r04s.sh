#!/bin/bash
# round 4, call s: GEMM tile-group size (M-tiles per raster group: 4 / 6 / 8) at the GEMM shapes and in the image
set -o pipefail
mkdir -p gpurun_out/r04s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd f-lite_amd
timeout -k 10 600 python -u tools/variants.py run gemm g_base g_grp4 g_grp8 --rounds 3 2>&1 | tee ../gpurun_out/r04s/variants.log | tail -5 || { echo "variants failed"; exit 1; }
cd ..
for v in g_base g_grp4 g_grp8 g_base g_grp4 g_grp8; do
  FLITE_LIB=$PWD/f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>&1 | tee -a gpurun_out/r04s/bench_$v.log | grep "^{" | cut -c1-120 || { echo "bench failed"; exit 1; }
done
