#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bh
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r05bh
timeout -k 5 20 amd-smi metric --power --clock --json > $out/smi_idle.json 2> $out/smi_err.txt || timeout -k 5 20 rocm-smi --showpower --showclocks --json > $out/smi_idle.json 2>>$out/smi_err.txt || true
timeout -k 10 300 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --negative-images 0 > $out/bench.log 2>&1 &
bp=$!
sleep 45
for i in $(seq 1 25); do
  echo "=== $(date +%s.%N)" >> $out/smi_samples.txt
  timeout -k 5 10 amd-smi metric --power --clock --json >> $out/smi_samples.txt 2>>$out/smi_err.txt || true
  sleep 0.5
done
wait $bp; rc=$?
tail -1 $out/bench.log | cut -c1-200
exit $rc
