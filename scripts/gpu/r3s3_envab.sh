#!/bin/bash
# whole-step A/B of an environment switch: $1 = tag, $2 = VAR, $3 = value A, $4 = value B, rest = bench.py args;
# order A B B A A B (cancels drift), one JSON per run
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="$1"; V="$2"; A="$3"; B="$4"; shift 4
cd "$R"; mkdir -p gpurun_out/$T
O="$R/gpurun_out/$T"
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for val in $A $B $B $A $A $B; do
  i=$((i+1))
  timeout -k 10 400 env $V=$val python bench.py "$@" > $O/run${i}_$val.log 2>&1 || { tail -5 $O/run${i}_$val.log; exit 1; }
  echo "$V=$val: $(grep -h '^{' $O/run${i}_$val.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
