#!/bin/bash
# round 5, call x: warp-specialised attention variants (priority, chained S halves): equality + timing
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_ATTN_Q256=0
L=f-lite_amd/tools/variants
timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump /tmp/old.pt > /tmp/eq.log 2>&1 || { tail -5 /tmp/eq.log; exit 1; }
for v in ws_chain ws_chain_sprio; do
  FLITE_ATTN_WS=1 FLITE_LIB=$L/$v/libflite_hip.so timeout -k 10 120 python -u f-lite_amd/tools/attn_equal.py dump /tmp/$v.pt >> /tmp/eq.log 2>&1 || { tail -5 /tmp/eq.log; exit 1; }
  echo "== $v equality"; timeout -k 10 60 python -u f-lite_amd/tools/attn_equal.py compare /tmp/$v.pt /tmp/old.pt 2>&1 | grep -c identical
done
for r in 1 2; do
  echo "== one-wave"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  echo "== ws"; FLITE_ATTN_WS=1 timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  for v in ws_sprio ws_oprio ws_chain ws_chain_sprio ws_chain_oprio; do
    echo "== $v"; FLITE_ATTN_WS=1 FLITE_LIB=$L/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  done
done
