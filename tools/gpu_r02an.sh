#!/usr/bin/env bash
# Round-2 GPU pass an: wide codes (40+8, 32+8) on the run-time kernels: workgroup size.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
{
  AB_K=40 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8" "op=rec8,bs_block=256" "jit=2" "bs_block=256" &&
  AB_K=24 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8" "op=rec8,bs_block=256" "op=rec8,jit=0" &&
  AB_K=10 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8" "op=rec8,jit=0"
} > "$OUT/ab_jit_wide2.log" 2>&1 || { tail -30 "$OUT/ab_jit_wide2.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_wide2.log"
