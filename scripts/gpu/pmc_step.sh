#!/bin/bash
# PMC counters over the whole GPT-2-small training step (bench.py), one pass per counter group:
# HBM bytes (TCC FETCH_SIZE / WRITE_SIZE) and SQ activity (MFMA busy, LDS conflicts) per kernel.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmcstep"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmcstep/p$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/pmcstep/p$i.log" 2>&1 || { echo "rocprof pass $i failed"; tail -5 "$R/gpurun_out/pmcstep/p$i.log"; exit 1; }
  echo "pass $i ok"
done
