#!/bin/bash
# round 5, call k: full GPU suite (incl. the 7B CFG-6 configs[1] floor and the full-size MXFP8 loop) + smoke,
# the 2-rank rehearsal bench line, and q256 stamps / DMA-placement variants
set -o pipefail
mkdir -p gpurun_out/r05k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05k/pytest.log 2>&1 || { tail -30 gpurun_out/r05k/pytest.log; exit 1; }
tail -3 gpurun_out/r05k/pytest.log
grep -E "PSNR|dB" gpurun_out/r05k/pytest.log | grep -E "30 steps|1024" | cut -c1-220 | tail -12
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05k/smoke.log 2>&1 || { tail -10 gpurun_out/r05k/smoke.log; exit 1; }
tail -2 gpurun_out/r05k/smoke.log
echo "== q256 stamps"
FLITE_LIB=f-lite_amd/tools/variants/q256stamps/libflite_hip.so timeout -k 10 200 python -u f-lite_amd/tools/attn_stamps_q256.py run > gpurun_out/r05k/stamps.log 2>&1 || { tail -5 gpurun_out/r05k/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05k/stamps.log | tail -12
for v in dmaburst dmaodd; do
  lib=f-lite_amd/tools/variants/$v/libflite_hip.so
  echo "== $v"
  FLITE_LIB=$lib timeout -k 10 120 python -u f-lite_amd/tools/q256_check.py 2>&1 | grep -E "q256:" | cut -c1-200 || exit 1
  FLITE_LIB=$lib timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self --rounds 2 2>&1 | grep -E "q256|q128" || exit 1
done
echo "== baseline"
timeout -k 10 200 python -u f-lite_amd/tools/q256_bench.py --shapes round,self --rounds 2 2>&1 | grep -E "q256|q128" || exit 1
FLITE_BENCH_REHEARSAL=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05k/rehearsal.log 2>&1 || { tail -10 gpurun_out/r05k/rehearsal.log; exit 1; }
tail -1 gpurun_out/r05k/rehearsal.log | cut -c1-400
