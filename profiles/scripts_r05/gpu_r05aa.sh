#!/bin/bash
# round 5, call aa: final build -- full GPU suite + smoke, and the BASELINE configs' bench lines
set -o pipefail
mkdir -p gpurun_out/r05aa
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
o=gpurun_out/r05aa
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -10 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --model 7b > $o/bench_7b.log 2>&1 || { tail -5 $o/bench_7b.log; exit 1; }
tail -1 $o/bench_7b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('7b 1024', d['value'], d.get('value_with_negative_prompt'))"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --height 896 --width 1344 --vae-tiling --negative-images 0 > $o/bench_1344.log 2>&1 || { tail -5 $o/bench_1344.log; exit 1; }
tail -1 $o/bench_1344.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1344 bf16', d['value'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --height 896 --width 1344 --vae-tiling --fp8 --negative-images 0 > $o/bench_fp8.log 2>&1 || { tail -5 $o/bench_fp8.log; exit 1; }
tail -1 $o/bench_fp8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1344 fp8', d['value'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || { tail -5 $o/bench.log; exit 1; }
tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('10b 1024', d['value'], d.get('value_with_negative_prompt'), d['roofline']['frac'])"
