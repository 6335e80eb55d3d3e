#!/bin/bash
# Same-lease image A/B of whole source trees (diagnostic; run on the GPU box from the repo root):
#   bash f-lite_amd/tools/bench_trees.sh OUT ROUNDS "BENCH ARGS" TREE...
# TREE "." is this tree; any other is a directory holding an older build's bench.py + f-lite_amd + oracle
# (e.g. abtrees/r2, made from a git worktree of that commit). Lines are tagged "== TREE ROUND" for
# tools/bench_ab_table.py.
out=$1; rounds=$2; args=$3; shift 3
root=$(pwd)
mkdir -p "$(dirname "$out")"
: > "$out"
for ((r = 1; r <= rounds; r++)); do
  for tree in "$@"; do
    echo "== $tree $r" >> "$out"
    (cd "$tree" && timeout -k 10 240 python -u bench.py $args) > "$root/$out.tmp" 2>&1 || { cat "$root/$out.tmp" >> "$out"; exit 1; }
    grep "^{" "$root/$out.tmp" >> "$out"
  done
done
rm -f "$out.tmp"
