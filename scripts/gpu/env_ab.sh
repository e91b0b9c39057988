#!/bin/bash
# Interleaved A/B of PLLM_AB settings on one box: the same bench.py command under each setting in turn.
# usage: SETTINGS="'' wt_shadow=0" bash scripts/gpu/env_ab.sh <tag> <rounds> <bench args...>
# ('' = defaults); one line per run is appended to gpurun_out/<tag>/env_ab.log as "ab=<setting> <json>"
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
eval "set -- $(printf '%q ' "$@")"
for r in $(seq 1 $ROUNDS); do
  for s in ${SETTINGS:-default}; do
    [ "$s" = default ] && ab="" || ab="$s"
    out=$(PLLM_AB="$ab" timeout -k 10 300 python bench.py "$@" 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$out" | grep '^{"metric' | sed "s|^|ab=$s |" >> $O/env_ab.log
  done
done
cut -c1-200 $O/env_ab.log
