#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05az
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rr in 1 2 4 1 2 4; do
  FLITE_NORM_RR=$rr timeout -k 10 120 python -u f-lite_amd/tools/norm_rr_check.py dump /tmp/rr$rr.pt 2>&1 | grep -v amdgpu.ids || exit 1
done
for rr in 2 4; do timeout -k 10 60 python -u f-lite_amd/tools/norm_rr_check.py compare /tmp/rr1.pt /tmp/rr$rr.pt || exit 1; done
