"""One wgrad shape, one kernel variant, N calls: a clean dispatch stream for rocprofv3 --pmc."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=65536)
ap.add_argument("--P", type=int, default=50304)
ap.add_argument("--Q", type=int, default=768)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--variants", default=None, help="comma-separated wgrad_set_mfma codes, run one after the other")
ap.add_argument("--calls", type=int, default=5)
a = ap.parse_args()
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()
dy = (torch.randn(a.M, a.P, device="cuda") * 0.1).bfloat16()
x = torch.randn(a.M, a.Q, device="cuda").bfloat16()
tgt = torch.zeros(a.P, a.Q, device="cuda")
for v in ([int(t) for t in a.variants.split(",")] if a.variants else [a.variant]):
    torch.ops.pllm.wgrad_set_mfma(v)
    for _ in range(a.calls):
        torch.ops.pllm.wgrad(dy, x, tgt)
torch.cuda.synchronize()
torch.ops.pllm.wgrad_set_mfma(0)
print("ok")
