#!/bin/bash
# round 6, call g: end-of-round evidence on the round-6 build: smoke, the default bench line (whole-step CPU
# baseline), a --no-graph kernel trace of the same workload, the gate/up counter passes (pmc_traffic.json), and
# counter passes for every kernel class with the bf16 residual (pmc_kernels.json)
set -o pipefail
out=gpurun_out/r06g
mkdir -p $out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash f-lite_amd/tools/round_evidence.sh $out > $out/evidence.log 2>&1 || { tail -20 $out/evidence.log; exit 1; }
tail -1 $out/evidence.log
python3 -c "
import json; d=json.load(open('$out/bench_line.json'))
print('value', d['value'], 'neg', d.get('value_with_negative_prompt'), 'frac', d['roofline']['frac'], 'util', d.get('mfma_util_image'), 'cpu', d['cpu_baseline']['value'], d['config']['residual_dtype'])"
python3 f-lite_amd/tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write $out/pmc_mfma $out/pmc_traffic.json > $out/pmc_traffic.log 2>&1 || { tail $out/pmc_traffic.log; exit 1; }
cat $out/pmc_traffic.json
