"""Fused softmax-CE kernel alone at the GPT-2 LM-head shape (65536 x 50304 bf16 logits, dlogits in
place), median microseconds over rounds; select an A/B build with PLLM_SO."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

N, V = 65536, 50304
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()
logits = (torch.randn(N, V, device="cuda") * 2).bfloat16()
tg = torch.randint(0, V, (N,), device="cuda")
inv = torch.tensor([1.0 / N], device="cuda")
for _ in range(3):
    torch.ops.pllm.cross_entropy(logits, tg, logits, -100, inv)
ts = []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        torch.ops.pllm.cross_entropy(logits, tg, logits, -100, inv)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) / 3 * 1e6)
print(f"ce {os.environ.get('PLLM_SO', 'in-tree')} median_us={statistics.median(ts):.1f} min_us={min(ts):.1f} "
      f"TB/s={2 * N * V * 2 / statistics.median(ts) / 1e6:.2f}", flush=True)
