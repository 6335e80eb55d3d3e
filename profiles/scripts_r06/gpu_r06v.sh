#!/bin/bash
# round 6, call v: end-of-round evidence on the final round-6 build (16-B-lane residual epilogues): smoke, the default bench line (whole-step CPU
# baseline), a --no-graph kernel trace of the same workload, the gate/up counter passes (pmc_traffic.json), and
# counter passes for every kernel class with the bf16 residual (pmc_kernels.json)
set -o pipefail
out=gpurun_out/r06v
mkdir -p $out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/round_evidence.sh $out > $out/evidence.log 2>&1 || { tail -20 $out/evidence.log; exit 1; }
tail -1 $out/evidence.log
python3 -c "
import json; d=json.load(open('$out/bench_line.json'))
print('value', d['value'], 'neg', d.get('value_with_negative_prompt'), 'frac', d['roofline']['frac'], 'util', d.get('mfma_util_image'), 'cpu', d['cpu_baseline']['value'], d['config']['residual_dtype'])"
python3 f-lite_amd/tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write $out/pmc_mfma $out/pmc_traffic.json > $out/pmc_traffic.log 2>&1 || { tail $out/pmc_traffic.log; exit 1; }
cat $out/pmc_traffic.json
K=f-lite_amd/tools/pmc_kernels.py
P=$out/pmck
mkdir -p $P
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $P/trace -o run -- python3 $K > $P/trace.log 2>&1 || { echo "trace failed"; tail $P/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $K > $P/fetch.log 2>&1 || { echo "fetch failed"; tail $P/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $K > $P/write.log 2>&1 || { echo "write failed"; tail $P/write.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/mfma -o run -- python3 $K > $P/mfma.log 2>&1 || { echo "mfma failed"; tail $P/mfma.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $P/stall -o run -- python3 $K > $P/stall.log 2>&1 || { echo "stall failed"; tail $P/stall.log; exit 1; }
python3 f-lite_amd/tools/pmc_reduce.py $P/pmc_kernels.json trace=$P/trace fetch=$P/fetch write=$P/write mfma=$P/mfma stall=$P/stall residual=bf16 > $P/reduce.log 2>&1 || { echo "reduce failed"; tail -20 $P/reduce.log; }
head -40 $P/reduce.log
tar czf $P/raw.tgz -C $P trace fetch write mfma stall && rm -rf $P/trace $P/fetch $P/write $P/mfma $P/stall
