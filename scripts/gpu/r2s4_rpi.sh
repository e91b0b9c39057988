#!/bin/bash
# GELU backward + column sums: full-row blocks (default build) vs 512-column panels (_C_panel.so) vs full rows, 8 rows per iteration (_C_rows8.so)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for so in panel rows8; do
  PLLM_SO=$R/pretraining_llm_amd/_C_$so.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "act or bias" --timeout 120 --timeout-method thread > gpurun_out/rpi_tests_$so.log 2>&1 || { tail -5 gpurun_out/rpi_tests_$so.log; exit 1; }
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "act or bias" --timeout 120 --timeout-method thread > gpurun_out/rpi_tests_base.log 2>&1 || { tail -5 gpurun_out/rpi_tests_base.log; exit 1; }
echo "variant tests ok"
cat > /tmp/gelu_mb.py <<'PY'
import sys, time, torch
sys.path.insert(0, ".")
from pretraining_llm_amd.ops import _lib
_lib.require()
N, C = 65536, 3072
x = torch.randn(N, C, device="cuda").bfloat16()
dy = torch.randn(N, C, device="cuda").bfloat16()
b = torch.zeros(C, device="cuda")
for _ in range(5):
    torch.ops.pllm.act_bwd_bias(dy, x, 1, b)
torch.cuda.synchronize()
best = 1e9
for _ in range(5):
    t0 = time.perf_counter()
    for _ in range(20):
        torch.ops.pllm.act_bwd_bias(dy, x, 1, b)
    torch.cuda.synchronize()
    best = min(best, (time.perf_counter() - t0) / 20)
print(f"act_bwd_bias gelu [65536x3072]: {best * 1e6:.1f} us ({3 * N * C * 2 / best / 1e12:.2f} TB/s)")
PY
for so in base panel rows8 base panel rows8; do
  if [ $so = base ]; then unset PLLM_SO; else export PLLM_SO=$R/pretraining_llm_amd/_C_$so.so; fi
  echo "$so: $(timeout -k 10 120 python /tmp/gelu_mb.py 2>&1 | tail -1)"
done
for so in base panel base panel; do
  if [ $so = base ]; then unset PLLM_SO; else export PLLM_SO=$R/pretraining_llm_amd/_C_$so.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/rows_bench_$so.log 2>&1 || { tail -5 gpurun_out/rows_bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 gpurun_out/rows_bench_$so.log | cut -c80-135)"
done
