#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu/r3_bstamps.sh && bash scripts/gpu/r3_attn_ab.sh "${1:-bwd1}" "${2:-}"
