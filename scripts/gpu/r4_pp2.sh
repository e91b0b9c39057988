#!/bin/bash
# ping-pong GEMM ablations (epilogue stores / main-loop DMA removed; wrong numerics by design) and
# counters of the kernel vs hipBLASLt
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/r4pp2
export HSA_ENABLE_IPC_MODE_LEGACY=0
for shape in "65536 3072 768" "32768 2048 2048"; do
  set -- $shape
  for round in 1 2; do
    for v in "" 1 2 3; do
      so=""; [ -n "$v" ] && so="$R/pretraining_llm_amd/_C_ppexp$v.so"
      PLLM_SO=$so timeout -k 10 120 python bench/gemm_one.py --M $1 --N $2 --K $3 --phased 4 --no-blas --time 2>&1 | grep median || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r4pp2"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
for shape in "3072 768" "768 3072"; do
  set -- $shape
  tag="N$1_K$2"; i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$O/${tag}_p$i" -o run --output-format csv -- \
      python3 "$R/bench/gemm_one.py" --N $1 --K $2 --phased 4 > "$O/${tag}_p$i.log" 2>&1 || { echo "pass $tag $i failed"; tail -5 "$O/${tag}_p$i.log"; exit 1; }
  done
  python3 "$R/scripts/pmc_kernels.py" "ping-pong TN GEMM vs hipBLASLt M=65536 N=$1 K=$2" "$O/${tag}_p1" "$O/${tag}_p2" > "$O/${tag}.md" || exit 1
  cat "$O/${tag}.md"
done
