#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u f-lite_amd/tools/attn_mixed_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== mix check"; FLITE_ATTN_MIX=1 timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:|q128:" | cut -c1-200 || exit 1
for r in 1 2; do
  echo "== auto"; timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes self,self1344 --rounds 2 2>&1 | grep -E "auto" || exit 1
  echo "== auto+mix"; FLITE_ATTN_MIX=1 timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes self,self1344 --rounds 2 2>&1 | grep -E "auto" || exit 1
done
