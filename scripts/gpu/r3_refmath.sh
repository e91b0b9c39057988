#!/bin/bash
# reference-algorithm baseline (materialised per-head attention) eager and torch.compile'd, vs this
# framework on the same architecture (preset ref-small) and on GPT-2 small
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/refmath
O=gpurun_out/refmath
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench/ref_math_bench.py --batch 64 --steps 5 --warmup 2 > $O/eager_b64.log 2>&1
rc=$?; tail -1 $O/eager_b64.log | cut -c1-400; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python bench.py --model ref-small --steps 10 --warmup 3 > $O/ours_refsmall.log 2>&1 || { tail -3 $O/ours_refsmall.log; exit 1; }
tail -1 $O/ours_refsmall.log | cut -c1-300
timeout -k 10 900 python bench/ref_math_bench.py --batch 64 --steps 5 --warmup 2 --compile > $O/compile_b64.log 2>&1
rc=$?; tail -1 $O/compile_b64.log | cut -c1-400; exit $rc
