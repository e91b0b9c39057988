#!/bin/bash
# bench.py default (hipGraph step auto-on at one GPU) vs --cuda-graph 0, plus the CLI/bench GPU tests
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/gdef
O="$R/gpurun_out/gdef"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_cli_gpu.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for v in default 0 default 0; do
  if [ $v = default ]; then F=; else F="--cuda-graph 0"; fi
  timeout -k 10 300 python bench.py $F > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  echo "$v: $(grep -h '^{' $O/b_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["cuda_graph"], d["steps"], d["warmup"])')"
done
