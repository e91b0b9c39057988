#!/bin/bash
# PMC passes over the wgrad kernels at the GPT-2 LM-head / fc shapes (variants 8 and 32)
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/wgpmc"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TA_TA_BUSY_sum"
for v in 8 32; do
  for shape in "50304 768" "3072 768"; do
    set -- $shape
    i=0
    for C in "$C1" "$C2"; do
      i=$((i+1))
      tag="v${v}_P$1_p$i"
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$O/$tag" -o run --output-format csv -- \
        python3 "$R/bench/wgrad_one.py" --P $1 --Q $2 --variant $v > "$O/$tag.log" 2>&1 || { echo "pass $tag failed"; tail -5 "$O/$tag.log"; exit 1; }
    done
    python3 "$R/scripts/pmc_kernels.py" "wgrad v$v P=$1 Q=$2 M=65536" "$O/v${v}_P$1_p1" "$O/v${v}_P$1_p2" > "$O/v${v}_P$1.md"
    grep -E "shares|MFMA busy|hit rate|duration" "$O/v${v}_P$1.md"
  done
done
