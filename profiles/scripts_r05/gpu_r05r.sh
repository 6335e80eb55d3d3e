#!/bin/bash
# round 5, call r: round evidence on the current build (smoke, default bench line with CPU baseline, --no-graph kernel
# trace, gate/up counter passes) + counter passes for every kernel class
set -o pipefail
mkdir -p gpurun_out/r05r
bash f-lite_amd/tools/round_evidence.sh gpurun_out/r05r > gpurun_out/r05r/evidence.log 2>&1 || { tail -20 gpurun_out/r05r/evidence.log; exit 1; }
tail -1 gpurun_out/r05r/evidence.log
python3 -c "
import json; d=json.load(open('gpurun_out/r05r/bench_line.json'))
print('value', d['value'], 'neg', d.get('value_with_negative_prompt'), 'frac', d['roofline']['frac'], 'util', d.get('mfma_util_image'), 'cpu', d['cpu_baseline']['value'])"
bash gpu_r05r_pmc.sh
