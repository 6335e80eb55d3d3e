#!/bin/bash
# round 5, call m: 256-row attention cycle anatomy, combined ablations (diagnostic builds: outputs not valid)
set -o pipefail
mkdir -p gpurun_out/r05m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in q256stamps st_mfmaonly st_mfma_smx st_nodma_nok st_mfma_dma; do
  echo "== $v"
  FLITE_LIB=f-lite_amd/tools/variants/$v/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run > gpurun_out/r05m/stamps_$v.log 2>&1 || { tail -5 gpurun_out/r05m/stamps_$v.log; exit 1; }
  grep -E "whole" gpurun_out/r05m/stamps_$v.log
done
