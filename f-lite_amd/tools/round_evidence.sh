#!/bin/bash
# End-of-round GPU evidence for the bench line (run on the GPU box from the repo root):
#   bash f-lite_amd/tools/round_evidence.sh OUTDIR
# smoke, the default bench line, a kernel trace (--stats) of the same workload without the hipGraph (rocprofv3
# segfaults tracing graph replays), and the gate/up GEMM's kernel-trace + three counter passes (FETCH_SIZE,
# WRITE_SIZE, MFMA set) over tools/pmc_gemm.py, each pass its own run (MI355X_MICROARCH.md, HBM/rocprofv3).
# Reduce the counter passes afterwards with tools/pmc_traffic.py.
set -e -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py > "$out/bench.log" 2>&1
grep "^{" "$out/bench.log" > "$out/bench_line.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --no-graph --steps 1 \
  --warmup 1 --no-cpu-baseline --probe none > "$out/trace.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/gemm_time" -o run -- python3 f-lite_amd/tools/pmc_gemm.py \
  > "$out/gemm_time.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python3 f-lite_amd/tools/pmc_gemm.py \
  > "$out/pmc_fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python3 f-lite_amd/tools/pmc_gemm.py \
  > "$out/pmc_write.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$out/pmc_mfma" -o run -- python3 f-lite_amd/tools/pmc_gemm.py > "$out/pmc_mfma.log" 2>&1
echo "round evidence done"
