#!/usr/bin/env bash
# Round-2 GPU pass ak: wide codes (40+8) on the run-time kernels: prefetch distance, vector size.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
{
  AB_K=40 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8,jit_pf=3" "op=rec8,jit_pf=5" "op=rec8,jit_pf=6" "op=rec8,jit_pf=2" &&
  AB_K=40 AB_M=8 AB_VEC=1048576 AB_ROUNDS=6 timeout -k 10 400 python -u tools/ab.py "op=rec8,jit_pf=3" "op=rec8,jit=0" "jit_pf=3" "jit=0"
} > "$OUT/ab_jit_wide.log" 2>&1 || { tail -30 "$OUT/ab_jit_wide.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_wide.log"
