#!/bin/bash
# round 5, call v: warp-specialised attention (FLITE_ATTN_WS=1) -- bit equality against the one-wave kernel, timing
set -o pipefail
mkdir -p gpurun_out/r05v
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_ATTN_Q256=0
FLITE_ATTN_WS=1 timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r05v/new.pt > gpurun_out/r05v/eq.log 2>&1 || { tail -5 gpurun_out/r05v/eq.log; exit 1; }
timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump gpurun_out/r05v/old.pt >> gpurun_out/r05v/eq.log 2>&1 || { tail -5 gpurun_out/r05v/eq.log; exit 1; }
timeout -k 10 60 python -u f-lite_amd/tools/attn_equal.py compare gpurun_out/r05v/new.pt gpurun_out/r05v/old.pt 2>&1 | tail -11 || exit 1
rm -f gpurun_out/r05v/*.pt
for r in 1 2; do
  echo "== ws"; FLITE_ATTN_WS=1 timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  echo "== one-wave"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
done
