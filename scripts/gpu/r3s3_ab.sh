#!/bin/bash
# generic A/B: in-tree _C.so ("new") vs pretraining_llm_amd/_C_base.so ("base"): $2 = pytest -k filter
# (file list $3, default tests/test_kernels_gpu.py), then the headline bench base/new x 2
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-ab}"
cd "$R"; mkdir -p gpurun_out/$T
O="$R/gpurun_out/$T"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest ${3:-tests/test_kernels_gpu.py} -q -x -k "${2:-wgrad}" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for so in base new base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench_$so.log 2>&1 || { tail -5 $O/bench_$so.log; exit 1; }
  echo "$so bench: $(grep -h '^{' $O/bench_$so.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
