#!/bin/bash
# Interleaved A/B of extension builds on one box: the same python command under each PLLM_SO in turn.
# usage: VARIANTS="base xso/a.so xso/b.so" bash scripts/gpu/ab.sh <tag> <rounds> <script.py> [args...]
# (base = the in-tree _C.so); one line per run is appended to gpurun_out/<tag>/ab.log as "so=<variant> <output>"
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then so=""; else so="$PWD/$v"; fi
    out=$(PLLM_SO=$so timeout -k 10 200 python "$@" 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$out" | grep -v amdgpu.ids | sed "s|^|so=$v |" >> $O/ab.log
  done
done
cat $O/ab.log
