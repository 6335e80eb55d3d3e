#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp FLITE_ATTN_Q256=0
L=f-lite_amd/tools/variants
for r in 1 2; do
  echo "== one-wave"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  for v in ws_chain wsc_k3 wsc_v6 wsc_k4v2; do
    echo "== $v"; FLITE_ATTN_WS=1 FLITE_LIB=$L/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self,cross --rounds 2 2>&1 | grep -E "q128" || exit 1
  done
done
