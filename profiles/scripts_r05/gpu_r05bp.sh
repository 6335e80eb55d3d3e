#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bp
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05bp/smoke.log 2>&1 || { tail -20 gpurun_out/r05bp/smoke.log; exit 1; }
tail -1 gpurun_out/r05bp/smoke.log
timeout -k 10 330 python -u bench.py > gpurun_out/r05bp/bench.log 2>&1 || { tail -20 gpurun_out/r05bp/bench.log; exit 1; }
python3 -c "import json; l=[x for x in open('gpurun_out/r05bp/bench.log') if x.startswith('{\"metric')][-1]; d=json.loads(l); print(d['value'], d['value_with_negative_prompt'], d['roofline']['frac'], d['cpu_baseline']['value'])"
