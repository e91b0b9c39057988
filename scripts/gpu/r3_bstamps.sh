#!/bin/bash
# backward attention phase stamps (diagnostic build xso/_C_bstamps.so)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/xso/_C_bstamps.so PLLM_BWD_STAMPS=1 timeout -k 10 120 python - <<'PY' 2>&1 | grep -v Warning | tail -8
import torch, math
from pretraining_llm_amd.ops import _lib
_lib.require()
for (B,H,T,D) in [(64,12,1024,64),(8,16,4096,64)]:
    q,k,v,do = (torch.randn(B,T,H,D,device="cuda",dtype=torch.bfloat16) for _ in range(4))
    o, lse = torch.ops.pllm.attn_fwd(q,k,v,True,1/math.sqrt(D))
    dq,dk,dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(3):
        torch.ops.pllm.attn_bwd(do,q,k,v,o,lse,dq,dk,dv,True,1/math.sqrt(D))
    torch.cuda.synchronize()
    print("cfg", B,H,T,D, flush=True)
PY
