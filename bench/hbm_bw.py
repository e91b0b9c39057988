"""HBM streaming ceiling on the box (1 GiB bf16 tensors, stock torch kernels): read+write copy,
write-only fill, read-only reduction.  The bandwidth-bound hand-written kernels (norms,
activations, fused cross-entropy, AdamW) are judged against these numbers
(profiles/r1_hbm_bandwidth.txt)."""
import time

import torch


def main():
    x = torch.empty(1 << 29, dtype=torch.bfloat16, device="cuda")  # 1 GiB
    y = torch.empty_like(x)
    x2 = torch.empty_like(x)
    x3 = torch.empty_like(x)
    for name, fn, nbytes in (("copy (read+write)", lambda: y.copy_(x), 2 * x.numel() * 2),
                             ("fill (write)", lambda: y.fill_(1.0), x.numel() * 2),
                             ("sum (read)", lambda: x.sum(), x.numel() * 2),
                             ("add (2 reads + write)", lambda: torch.add(x, x2, out=y), 3 * x.numel() * 2),
                             ("addcmul (3 reads + write)", lambda: torch.addcmul(x, x2, x3, out=y), 4 * x.numel() * 2)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 20
        print(f"{name}: {nbytes / dt / 1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
