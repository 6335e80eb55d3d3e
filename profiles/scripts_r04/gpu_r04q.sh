#!/bin/bash
# round 4, call q: attention read-ahead depths on the round-4 loop (V^T reads 2/4/6 MFMAs ahead, K reads 3/5 k-steps)
set -o pipefail
mkdir -p gpurun_out/r04q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd f-lite_amd
VARIANTS_CHECK=1 timeout -k 10 600 python -u tools/variants.py run attention a_base a_va6 a_va2 a_ka5 --rounds 3 2>&1 | tee ../gpurun_out/r04q/variants.log | tail -12 || { echo "variants failed"; exit 1; }
