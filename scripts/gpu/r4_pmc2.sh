#!/bin/bash
# counter passes of the current ping-pong TN GEMM vs hipBLASLt, and of the ping-pong vs one-barrier wgrad
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/pmc2"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
for shape in "768 3072" "3072 768"; do
  set -- $shape
  tag="N$1_K$2"
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$O/${tag}_p$i" -o run --output-format csv -- \
      python3 "$R/bench/gemm_one.py" --N $1 --K $2 --phased 4 > "$O/${tag}_p$i.log" 2>&1 || { echo "pass $tag $i failed"; tail -5 "$O/${tag}_p$i.log"; exit 1; }
  done
  python3 "$R/scripts/pmc_kernels.py" "ping-pong TN GEMM (round-4 final) vs hipBLASLt M=65536 N=$1 K=$2" "$O/${tag}_p1" "$O/${tag}_p2" > "$O/${tag}.md" || exit 1
  grep -E "^## |MFMA busy" "$O/${tag}.md" | grep -v "0.0%" | grep -B1 "MFMA busy"
done
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$O/wg_p$i" -o run --output-format csv -- \
    python3 "$R/bench/wgrad_one.py" --M 65536 --P 50304 --Q 768 --variants 0,100 > "$O/wg_p$i.log" 2>&1 || { echo "wgrad pass $i failed"; tail -5 "$O/wg_p$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_kernels.py" "wgrad M=65536 P=50304 Q=768: ping-pong (wgrad_pp_kernel) vs one-barrier (wgrad_kernel)" "$O/wg_p1" "$O/wg_p2" > "$O/wg.md" || exit 1
grep -E "^## |MFMA busy" "$O/wg.md" | grep -B1 "MFMA busy" | grep -v "0.0%"
