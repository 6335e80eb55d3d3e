#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05g
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
echo "== q256 stamps"
FLITE_LIB=f-lite_amd/tools/variants/q256stamps/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run 2>&1 | grep -v amdgpu.ids || exit 1
echo "== q128 stamps"
FLITE_LIB=f-lite_amd/tools/variants/stamps/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps.py run 2>&1 | grep -v amdgpu.ids || exit 1
