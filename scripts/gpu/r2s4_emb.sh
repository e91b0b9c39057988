#!/bin/bash
# skew-robust embedding backward: numerics (uniform / Zipf / chunk-boundary runs / one id), then
# the Trainer at the bench config on the Zipf-like Markov shard, then the headline bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "embedding" --timeout 120 --timeout-method thread > gpurun_out/emb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/emb_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python - <<'PY' > gpurun_out/emb_bench.log 2>&1 || { tail -5 gpurun_out/emb_bench.log; exit 2; }
import torch, time, sys
sys.path.insert(0, ".")
from pretraining_llm_amd.ops import _lib
_lib.require()
V, C, B, T = 50304, 768, 64, 1024
N = B * T
dx = torch.randn(B, T, C, device="cuda").bfloat16()
g = torch.zeros(V, C, device="cuda")
for kind in ("uniform", "zipf", "single"):
    if kind == "uniform":
        idx = torch.randint(0, V, (B, T), device="cuda")
    elif kind == "zipf":
        z = torch.distributions.Pareto(1.0, 0.3).sample((N,)).floor().long() - 1
        idx = (z.clamp_max(V - 1) * 7919 % V).view(B, T).cuda()
    else:
        idx = torch.full((B, T), 5, device="cuda")
    top = torch.bincount(idx.view(-1)).max().item()
    for _ in range(3):
        torch.ops.pllm.embedding_bwd_acc(dx, idx, V, 0, False, g)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(20):
        torch.ops.pllm.embedding_bwd_acc(dx, idx, V, 0, False, g)
    torch.cuda.synchronize()
    print(f"{kind}: largest run {top}, {1e6 * (time.perf_counter() - t0) / 20:.1f} us per call (incl. sort)")
PY
cat gpurun_out/emb_bench.log
timeout -k 10 400 python scripts/train_transformer.py --preset=gpt2-small --t_batch_size=64 --t_train_steps=41 \
  --t_eval_steps=1000 --eval_at_start=False --log_interval=10 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn \
  --t_out_path=None > gpurun_out/s4_trainer2.log 2>&1 || { echo "trainer failed"; tail -20 gpurun_out/s4_trainer2.log; exit 3; }
grep -E "Step" gpurun_out/s4_trainer2.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s4_bench_e.log 2>&1 || { tail -5 gpurun_out/s4_bench_e.log; exit 4; }
tail -1 gpurun_out/s4_bench_e.log | cut -c1-200
