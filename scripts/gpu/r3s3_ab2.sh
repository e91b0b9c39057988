#!/bin/bash
# A/B where "new" is an alternative build selected by PLLM_SO ($2, e.g. pretraining_llm_amd/_C_unroll.so) and
# "base" the in-tree _C.so: kernel GPU tests (-k $3) on the new build, then the headline bench base/new x 2
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-ab2}"; NEW="$R/$2"
cd "$R"; mkdir -p gpurun_out/$T
O="$R/gpurun_out/$T"
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$NEW timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "${3:-wgrad}" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for so in base new base new; do
  if [ $so = new ]; then export PLLM_SO=$NEW; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$so.log 2>&1 || { tail -5 $O/bench_$so.log; exit 1; }
  echo "$so bench: $(grep -h '^{' $O/bench_$so.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
