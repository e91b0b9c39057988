#!/bin/bash
# elementwise-kernel launch / unroll / nontemporal variants (xso/) vs shipped, HBM probe
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for v in cur $(ls xso | sed -e 's/^_C_//' -e 's/\.so$//'); do
    so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
    echo "$round $v $(PLLM_SO=$so timeout -k 10 120 python bench/hbm_probe.py 2>&1 | grep '^{')"
  done
done
