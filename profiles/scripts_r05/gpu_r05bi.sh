#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05bi
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r05bi
timeout -k 5 20 amd-smi list --json > $out/smi_list.json 2> $out/smi_err.txt || true
timeout -k 10 300 python -u bench.py --steps 12 --warmup 1 --no-cpu-baseline --negative-images 0 > $out/bench.log 2>&1 &
bp=$!
for i in $(seq 1 200); do
  kill -0 $bp 2>/dev/null || break
  echo "=== $(date +%s.%N)" >> $out/smi_samples.txt
  timeout -k 5 10 amd-smi metric --power --clock --json >> $out/smi_samples.txt 2>>$out/smi_err.txt || true
  sleep 0.3
done
wait $bp; rc=$?
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('torch device', p.name, getattr(p,'pci_bus_id',None), getattr(p,'pci_device_id',None))" >> $out/torch_dev.txt 2>&1 || true
tail -1 $out/bench.log | cut -c1-160
exit $rc
