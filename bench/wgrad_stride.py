"""Weight gradient of llama's down projection, dW[2048, 5504] = dY[M, 2048]^T X[M, 5504], with X's row stride
5504 (contiguous, 11008-B rows) vs padded to 5632 / 5568 (a column view of a wider buffer); plus the same for
the up-projection data gradient's operand.  Median microseconds, interleaved."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pretraining_llm_amd.ops import _lib  # noqa: E402
P = _lib.require()
from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402
enable_tuned_gemms(0)


def once(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


M, C, Fh = 32768, 2048, 5504
dy = (torch.randn(M, C, device="cuda") * 0.1).bfloat16()
w_down = (torch.randn(C, Fh, device="cuda") * Fh ** -0.5).bfloat16()
xs = {}
for ld in (5504, 5568, 5632, 6144):
    buf = torch.randn(M, ld, device="cuda").bfloat16()
    xs[ld] = buf[:, :Fh]
tgt = torch.zeros(C, Fh, device="cuda")
fns = {}
for ld, x in xs.items():
    fns[f"wgrad_ld{ld}"] = (lambda x=x: P.wgrad(dy, x, tgt))
    fns[f"down_fwd_ld{ld}"] = (lambda x=x: F.linear(x, w_down))
for f in fns.values():
    f(), f()
ts = {k: [] for k in fns}
for _ in range(7):
    for k, f in fns.items():
        ts[k].append(once(f))
print(json.dumps({k: round(statistics.median(v), 1) for k, v in ts.items()}), flush=True)
