#!/bin/bash
# PMC counters (SQ block) for the attention kernels at the GPT-2-small shape.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES"
for only in bwd fwd; do
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmc/${only}$i" -o run --output-format csv -- \
      python3 "$R/bench/attn_bench.py" --configs 64x12x1024x64 --only $only > "$R/gpurun_out/pmc/${only}$i.log" 2>&1 || { echo "rocprof $only $i failed"; tail -5 "$R/gpurun_out/pmc/${only}$i.log"; exit 1; }
  done
done
echo done
