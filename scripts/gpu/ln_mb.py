"""LayerNorm(+residual) forward microbench at the GPT-2-small shape (65536 x 768)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from pretraining_llm_amd.ops import _lib  # noqa: E402

_lib.require()
N, C = 65536, 768
x = torch.randn(N, C, device="cuda").bfloat16()
r = torch.randn(N, C, device="cuda").bfloat16()
w = torch.randn(C, device="cuda").bfloat16()
b = torch.randn(C, device="cuda").bfloat16()
for _ in range(5):
    torch.ops.pllm.norm_fwd(x, r, w, b, 1e-5, False)
torch.cuda.synchronize()
best = 1e9
for _ in range(5):
    t0 = time.perf_counter()
    for _ in range(50):
        torch.ops.pllm.norm_fwd(x, r, w, b, 1e-5, False)
    torch.cuda.synchronize()
    best = min(best, (time.perf_counter() - t0) / 50)
print(f"norm_fwd+res [65536x768]: {best * 1e6:.1f} us ({4 * N * C * 2 / best / 1e12:.2f} TB/s)")
