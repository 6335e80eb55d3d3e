#!/bin/bash
# round 4, call n: counter passes for every kernel class (attention refresh; collapse-shape cross-attention)
set -o pipefail
out=gpurun_out/r04n
mkdir -p $out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K=f-lite_amd/tools/pmc_kernels.py
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 $K > $out/trace.log 2>&1 || { echo "trace failed"; tail $out/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 $K > $out/fetch.log 2>&1 || { echo "fetch failed"; tail $out/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 $K > $out/write.log 2>&1 || { echo "write failed"; tail $out/write.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/mfma -o run -- python3 $K > $out/mfma.log 2>&1 || { echo "mfma failed"; tail $out/mfma.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $out/stall -o run -- python3 $K > $out/stall.log 2>&1 || { echo "stall failed"; tail $out/stall.log; exit 1; }
python3 f-lite_amd/tools/pmc_reduce.py $out/pmc_kernels.json trace=$out/trace fetch=$out/fetch write=$out/write mfma=$out/mfma stall=$out/stall > $out/reduce.log 2>&1 || { echo "reduce failed"; tail -20 $out/reduce.log; }
cat $out/reduce.log | head -60
tar czf $out/raw.tgz -C $out trace fetch write mfma stall && rm -rf $out/trace $out/fetch $out/write $out/mfma $out/stall
