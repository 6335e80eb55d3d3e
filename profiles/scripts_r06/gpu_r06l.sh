#!/bin/bash
# round 6, call l: MXFP8 policies at the BASELINE row's CFG 6 against the reference (VERDICT r05 missing 2): which
# per-block mixes reach the reference's own bf16 floor (10B 28.33 / 7B 27.37 dB at 1024^2), and their speed
set -o pipefail
mkdir -p gpurun_out/r06l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P="bf16|0-7:none|0-15:none|0-23:none|0-7:none;8-39:down|0-7:none;8-39:gate_up|0-7:none;8-39:gate_up+down|0-15:none;16-39:gate_up+down|0-3:none;4-39:down|all"
timeout -k 10 900 python -u f-lite_amd/tools/fp8_block_policy.py --cfg 6 --policies "$P" > gpurun_out/r06l/fp8_block_policy_cfg6.log 2>&1 || { tail -20 gpurun_out/r06l/fp8_block_policy_cfg6.log; exit 1; }
grep '^{' gpurun_out/r06l/fp8_block_policy_cfg6.log
run() {  # name, args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --negative-images 0 --probe none $2 > gpurun_out/r06l/bench_$1.log 2>&1 || { tail -5 gpurun_out/r06l/bench_$1.log; exit 1; }
  tail -1 gpurun_out/r06l/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
run bf16 ""
run fp8_0-15 "--fp8 --fp8-block-classes 0-15:none"
run fp8_0-7_down "--fp8 --fp8-block-classes 0-7:none;8-39:down"
run fp8_0-7_gu "--fp8 --fp8-block-classes 0-7:none;8-39:gate_up"
run fp8_0-7_gud "--fp8 --fp8-block-classes 0-7:none;8-39:gate_up+down"
