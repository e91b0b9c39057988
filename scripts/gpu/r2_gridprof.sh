#!/bin/bash
# per-kernel times of the GPT-2 step: full-grid build (cur) vs xso/_C_head.so
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
for v in cur head; do
  so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
  PLLM_SO=$so bash scripts/gpu/prof.sh r2_gridprof_$v --steps 5 --warmup 3 > /dev/null 2>&1 || { echo "prof $v failed"; exit 1; }
  python scripts/prof_summary.py gpurun_out/r2_gridprof_$v/run_kernel_stats.csv 8 "GPT-2 $v" > gpurun_out/r2_gridprof_$v.md
done
python3 - <<'PY'
import re
def load(p):
    d={}
    for l in open(p):
        if l.startswith('| ') and '`' in l:
            parts=[x.strip() for x in l.strip().strip('|').split('|')]
            try: d[parts[4][:60]]=float(parts[0])
            except: pass
    return d
a=load('gpurun_out/r2_gridprof_cur.md'); b=load('gpurun_out/r2_gridprof_head.md')
for k in sorted(set(a)|set(b), key=lambda k:-(a.get(k,0)+b.get(k,0)))[:22]:
    print(f"{a.get(k,0):8.3f} {b.get(k,0):8.3f} {a.get(k,0)-b.get(k,0):+7.3f}  {k}")
PY
