#!/bin/bash
# PMC passes over the attention kernels: llama shape (D=128) and GPT-2 shape (D=64)
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/attnpmc3"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAVES"
C3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for cfg in 64x12x1024x64 16x16x2048x128; do
  for only in fwd bwd; do
    i=0
    for C in "$C1" "$C2" "$C3"; do
      i=$((i+1))
      tag="${cfg}_${only}_p$i"
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$O/$tag" -o run --output-format csv -- \
        python3 "$R/bench/attn_bench.py" --configs $cfg --only $only --rounds 1 > "$O/$tag.log" 2>&1 || { echo "pass $tag failed"; tail -5 "$O/$tag.log"; exit 1; }
    done
    python3 "$R/scripts/pmc_kernels.py" "attention $only $cfg" "$O/${cfg}_${only}_p1" "$O/${cfg}_${only}_p2" "$O/${cfg}_${only}_p3" > "$O/${cfg}_${only}.md"
  done
done
echo done
