#!/bin/bash
# kernel-trace resource columns + counter passes: hand-written TN GEMM vs hipBLASLt at two shapes
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/gemmpmc"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
for shape in "768 3072" "3072 768"; do
  set -- $shape
  tag="N$1_K$2"
  timeout -s KILL 90 rocprofv3 --kernel-trace -d "$O/${tag}_kt" -o run --output-format csv -- \
    python3 "$R/bench/gemm_one.py" --N $1 --K $2 > "$O/${tag}_kt.log" 2>&1 || { echo "kt $tag failed"; tail -5 "$O/${tag}_kt.log"; exit 1; }
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$O/${tag}_p$i" -o run --output-format csv -- \
      python3 "$R/bench/gemm_one.py" --N $1 --K $2 > "$O/${tag}_p$i.log" 2>&1 || { echo "pass $tag $i failed"; tail -5 "$O/${tag}_p$i.log"; exit 1; }
  done
  python3 "$R/scripts/pmc_kernels.py" "TN GEMM vs hipBLASLt M=65536 N=$1 K=$2" "$O/${tag}_p1" "$O/${tag}_p2" > "$O/${tag}.md" || exit 1
  f=$(ls $O/${tag}_kt/*kernel_trace.csv | head -1)
  python3 - "$f" <<'PY'
import csv, sys
seen = set()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:70]
    if k in seen:
        continue
    seen.add(k)
    print(k, {c: r.get(c) for c in ("Workgroup_Size", "Grid_Size", "LDS_Block_Size", "Arch_VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")})
PY
done
