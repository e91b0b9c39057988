#!/bin/bash
# attention A/B (r3_attn_ab.sh) + a bank-conflict counter pass over the D=64 backward
R="${GRAFT_REPO_ROOT:-/root/repo}"
bash "$R/scripts/gpu/r3_attn_ab.sh" "$@" || exit 1
O="$R/gpurun_out/$1"
cd /tmp && export TMPDIR=/tmp
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C2 -d "$O/pmc" -o run --output-format csv -- \
  python3 "$R/bench/attn_bench.py" --configs 16x16x2048x128 --only bwd --rounds 1 > "$O/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$O/pmc.log"; exit 1; }
python3 "$R/scripts/pmc_kernels.py" "attention bwd 16x16x2048x128 (ImgS dS^T)" "$O/pmc" > "$O/pmc.md"
grep -A12 "attn_bwd_rs_kernel" "$O/pmc.md" | grep -E "BANK|INSTS_LDS|duration|MFMA busy"
