#!/bin/bash
# One parameterised driver for every GPU-box job (replaces the per-round r*_*.sh one-offs).
#
# usage: bash scripts/gpu/run.sh <out-tag> <task> [<task> ...]
# Tasks run in order; the first failure ends the call (no GPU step after a fault / timeout).
#   tests                 GPU test suite (pytest -m gpu)
#   tests:<expr>          GPU tests selected by pytest -k <expr>
#   smoke                 __graft_entry__.smoke()
#   bench:<name>[:args]   python bench.py <args>; no args: the named config (CFG below), else '+'-separated
#                         literal args, e.g. bench:llama or bench:l8:--model+llama-1.3b+--batch+8
#   prof:<name>[:args]    rocprofv3 kernel trace + stats of bench.py <args> (same rule), summarised to <name>.md
#   pmc:<name>:<counterset>:<script>[:args]
#                         one rocprofv3 --pmc pass per counter set group (see SETS below) over
#                         python3 <script> <args>, summarised by scripts/pmc_kernels.py to <name>.md
#   py:<name>:<script>[:args]   python3 <script> <args> > <name>.log
# Named configs: llama = --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2, etc. (CFG below)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
cd "$R"

declare -A CFG=(
  [gpt2]=""
  [llama]="--model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2"
  [ref3b]="--model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2"
  [medium]="--model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 5 --warmup 2"
  [gpt2prof]="--steps 8 --warmup 3"
  [llamaprof]="--model llama-1.3b --batch 16 --seq 2048 --steps 3 --warmup 2"
  [mediumprof]="--model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 3 --warmup 2"
)
# counter sets: each fits one pass (<= 8 SQ, <= 4 TCC, <= 2 GRBM)
declare -A SETS=(
  [core]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
  [inst]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAVES"
  [mem]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
)

args_of() {  # named config or '+'-separated literal args
  local a="$1"
  if [ -n "$a" ] && [ -n "${CFG[$a]+x}" ]; then echo "${CFG[$a]}"; else echo "${a//+/ }"; fi
}

for task in "$@"; do
  IFS=':' read -r kind name rest <<< "$task"
  case "$kind" in
    tests)
      sel=(); [ -n "$name" ] && sel=(-k "$name")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" \
        > "$O/tests.log" 2>&1
      rc=$?; grep -E "FAILED|passed|failed|error" "$O/tests.log" | tail -8; [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { tail -5 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python bench.py $(args_of "${rest:-$name}") > "$O/bench_$name.log" 2>&1 \
        || { tail -3 "$O/bench_$name.log"; exit 1; }
      tail -1 "$O/bench_$name.log" | cut -c1-260 ;;
    prof)
      a=$(args_of "${rest:-$name}")
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
          python3 "$R/bench.py" $a > "$O/$name.log" 2>&1 ) || { tail -3 "$O/$name.log"; exit 1; }
      steps=$(python3 -c "import sys,json; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][-1]); print(d['steps']+d['warmup']+(2 if d.get('config', {}).get('step_mode')=='graph' else 0))" "$O/$name.log") || exit 1
      # (graph mode: GraphedTrainStep runs 2 eager warm-up steps before its capture, bench.py:199)
      python3 scripts/prof_summary.py "$O/$name/run_kernel_stats.csv" "$steps" "$name: bench.py $a" > "$O/$name.md" || exit 1
      head -14 "$O/$name.md" ;;
    pmc)
      IFS=':' read -r sets script sargs <<< "$rest"
      dirs=()
      for s in ${sets//+/ }; do
        ( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${SETS[$s]} -d "$O/${name}_$s" -o run \
            --output-format csv -- python3 "$R/$script" ${sargs//+/ } > "$O/${name}_$s.log" 2>&1 ) \
          || { echo "pmc $name $s failed"; tail -5 "$O/${name}_$s.log"; exit 1; }
        dirs+=("$O/${name}_$s")
      done
      python3 scripts/pmc_kernels.py "$name: $script ${sargs//+/ }" "${dirs[@]}" > "$O/$name.md" || exit 1
      grep -E "^## |MFMA busy|shares" "$O/$name.md" | head -30 ;;
    ktrace)  # kernel trace + stats of a script: ktrace:<name>:<script>[:args]
      IFS=':' read -r script sargs <<< "$rest"
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
          python3 "$R/$script" ${sargs//+/ } > "$O/$name.log" 2>&1 ) || { tail -5 "$O/$name.log"; exit 1; }
      python3 scripts/prof_summary.py "$O/$name/run_kernel_stats.csv" 1 "$name: $script ${sargs//+/ }" > "$O/$name.md" || exit 1
      head -14 "$O/$name.md" ;;
    py)
      IFS=':' read -r script sargs <<< "$rest"
      timeout -k 10 600 python3 -u "$script" ${sargs//+/ } > "$O/$name.log" 2>&1 || { tail -5 "$O/$name.log"; exit 1; }
      tail -6 "$O/$name.log" ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "run.sh $TAG: all tasks ok"
