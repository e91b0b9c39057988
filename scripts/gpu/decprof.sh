#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/decprof"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/decprof" -o run --output-format csv -- \
  python3 "$R/bench/decode_prof.py" --batch 1 --new 64 --graph 0 > "$R/gpurun_out/decprof/log.txt" 2>&1
echo "rc=$?"; tail -2 "$R/gpurun_out/decprof/log.txt"
