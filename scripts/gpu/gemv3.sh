#!/bin/bash
# decode skinny-GEMM kernel: numerics tests, decode bench, decode-step kernel profile
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/decprof9
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemv or decode or generate or sampling" > gpurun_out/g8.log 2>&1
rc=$?; tail -2 gpurun_out/g8.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/g8.log | head -30; exit $rc; fi
timeout -k 10 300 python bench/decode_bench.py > gpurun_out/g8_dec.jsonl 2>gpurun_out/g8_dec.err || { tail -20 gpurun_out/g8_dec.err; exit 4; }
cat gpurun_out/g8_dec.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/decprof9" -o run --output-format csv -- \
  python3 "$R/bench/decode_prof.py" --batch 1 --new 64 --graph 1 > "$R/gpurun_out/decprof9/log.txt" 2>&1
echo "rc=$?"
