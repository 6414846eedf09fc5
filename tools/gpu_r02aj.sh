#!/usr/bin/env bash
# Round-2 GPU pass aj: run-time kernels over up to 64 columns (tests, A/B on wide codes).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/aj_pytest_jit.log" 2>&1 || { tail -60 "$OUT/aj_pytest_jit.log"; exit 1; }
tail -1 "$OUT/aj_pytest_jit.log"
{
  AB_K=40 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8,jit=0" "op=rec8,jit=2" "jit=0" "jit=2" &&
  AB_K=48 AB_M=16 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec16,jit=0" "op=rec16,jit=2"
} > "$OUT/ab_jit64.log" 2>&1 || { tail -30 "$OUT/ab_jit64.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit64.log"
