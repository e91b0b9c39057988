#!/bin/bash
# wgrad stage-loop phase stamps (diagnostic build xso/_C_wstamps.so)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/xso/_C_wstamps.so PLLM_WGRAD_STAMPS=1 timeout -k 10 120 python - <<'PY' 2>&1 | grep -v Warning | tail -12
import torch
from pretraining_llm_amd.ops import _lib
_lib.require()
for (M,P,Q) in [(65536,50304,768),(65536,3072,768),(65536,768,3072),(65536,2304,768),(32768,11008,2048),(32768,50304,2048)]:
    dy = torch.randn(M,P,device="cuda",dtype=torch.bfloat16)
    x = torch.randn(M,Q,device="cuda",dtype=torch.bfloat16)
    out = torch.zeros(P,Q,device="cuda",dtype=torch.float32)
    torch.ops.pllm.wgrad(dy, x, out)
    torch.cuda.synchronize()
    del dy, x, out
PY
