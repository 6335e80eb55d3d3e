#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=f-lite_amd/tools/variants
T="import sys; sys.path.insert(0,'f-lite_amd/tools'); import variants; r=variants.time_gemms(); print({k:(round(v[0]*1e3,1), round(v[1]/2516.6,3)) for k,v in r.items()})"
for r in 1 2; do
  echo "== grp6 (product)"; timeout -k 10 200 python -u -c "$T" 2>&1 | grep -v amdgpu.ids || exit 1
  for v in grp2 grp3 grp12 grp33; do
    echo "== $v"; FLITE_LIB=$L/$v/libflite_hip.so timeout -k 10 200 python -u -c "$T" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
