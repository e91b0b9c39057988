#!/bin/bash
# Interleaved A/B of two source trees on one box: bench.py from the repo root and from <other tree>, in turn.
# usage: bash scripts/gpu/tree_ab.sh <tag> <rounds> <other tree> [bench args...]
set -o pipefail
TAG=$1; ROUNDS=$2; OTHER=$3; shift 3
O=$PWD/gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for t in . "$OTHER"; do
    out=$(cd "$t" && timeout -k 10 300 python bench.py "$@" 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$out" | grep '^{"metric' | sed "s|^|tree=$t |" >> $O/tree_ab.log
  done
done
cut -c1-160 $O/tree_ab.log
