export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $GRAFT_REPO_ROOT
for so in v3qb1w2 v3qb1w3; do PLLM_SO=$GRAFT_REPO_ROOT/xso/_C_$so.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attn or attention or flash" --timeout 120 --timeout-method thread > gpurun_out/t_$so.log 2>&1; echo "$so $(tail -1 gpurun_out/t_$so.log)"; done
bash scripts/gpu/r3_attn_abl.sh
