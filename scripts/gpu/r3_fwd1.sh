#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu/r3_stamps.sh && bash scripts/gpu/r3_attn_ab.sh "${1:-fwd1}" "${2:-}"
