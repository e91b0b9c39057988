#!/bin/bash
# Kernel-level profile of the 1-GPU headline bench: rocprofv3 kernel trace + stats.
# usage: bash scripts/gpu/prof.sh <tag> [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-prof}; shift
mkdir -p "$R/gpurun_out/$TAG"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" "$@" > "$R/gpurun_out/$TAG/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 "$R/gpurun_out/$TAG/bench.log"
exit $rc
