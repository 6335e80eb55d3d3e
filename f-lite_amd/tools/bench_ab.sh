#!/bin/bash
# Same-box image-level A/B of library builds (diagnostic; run on the GPU box from the repo root):
#   bash f-lite_amd/tools/bench_ab.sh OUT ROUNDS "BENCH ARGS" SPEC...
# SPEC = NAME[:VAR=VALUE]; NAME "prod" is the in-tree product library, any other name a tools/variants/NAME build.
# Variants alternate within each round; every bench.py line goes to OUT, tagged "== SPEC ROUND".
out=$1; rounds=$2; args=$3; shift 3
mkdir -p "$(dirname "$out")"
: > "$out"
for ((r = 1; r <= rounds; r++)); do
  for spec in "$@"; do
    name=${spec%%:*}
    envkv=""
    [[ $spec == *:* ]] && envkv=${spec#*:}
    if [[ $name == prod ]]; then lib=f-lite_amd/f_lite/libflite_hip.so; else lib=f-lite_amd/tools/variants/$name/libflite_hip.so; fi
    echo "== $spec $r" >> "$out"
    if [[ -n $envkv ]]; then
      env "$envkv" FLITE_LIB="$lib" timeout -k 10 240 python -u bench.py $args > "$out.tmp" 2>&1 || { cat "$out.tmp" >> "$out"; exit 1; }
    else
      FLITE_LIB="$lib" timeout -k 10 240 python -u bench.py $args > "$out.tmp" 2>&1 || { cat "$out.tmp" >> "$out"; exit 1; }
    fi
    grep "^{" "$out.tmp" >> "$out"
  done
done
rm -f "$out.tmp"
