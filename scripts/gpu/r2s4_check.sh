#!/bin/bash
# session-4 re-entry check: GPU suite, smoke and the headline bench on the rebuilt tree, then a
# probe of two RCCL ranks sharing the one GPU (to rehearse the multi-rank bench on RCCL itself)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s4_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/s4_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 || { tail -5 gpurun_out/s4_smoke.log; exit 1; }
tail -1 gpurun_out/s4_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/s4_gpt2.log 2>&1 || { tail -5 gpurun_out/s4_gpt2.log; exit 1; }
tail -1 gpurun_out/s4_gpt2.log | cut -c1-400
timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/gpu/r2_rccl_probe.py > gpurun_out/s4_rccl_probe.log 2>&1
echo "rccl probe rc=$?"; tail -8 gpurun_out/s4_rccl_probe.log | cut -c1-300
exit 0
