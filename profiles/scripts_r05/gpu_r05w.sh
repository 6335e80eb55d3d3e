#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_ATTN_Q256=0
echo "== ws"; FLITE_ATTN_WS=1 timeout -k 10 120 python -u f-lite_amd/tools/ws_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
FLITE_ATTN_WS=1 timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump /tmp/new.pt > gpurun_out/r05w/eq.log 2>&1 || { tail -5 gpurun_out/r05w/eq.log; exit 1; }
timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump /tmp/old.pt >> gpurun_out/r05w/eq.log 2>&1 || { tail -5 gpurun_out/r05w/eq.log; exit 1; }
timeout -k 10 60 python -u f-lite_amd/tools/attn_equal.py compare /tmp/new.pt /tmp/old.pt 2>&1 | tail -11
for r in 1 2; do
  echo "== ws"; FLITE_ATTN_WS=1 timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  echo "== one-wave"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
done
