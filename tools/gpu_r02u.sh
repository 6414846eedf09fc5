#!/usr/bin/env bash
# Round-2 GPU pass u: run-time bit-sliced kernels (jit.cpp): parity tests, then
# same-process A/B against the perm-table kernels (10+8 Reconst of 5 / 6 / 8,
# 16+8 Encode, 10+8 Update / Replace).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
echo "== jit tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/u_pytest_jit.log" 2>&1 || { tail -60 "$OUT/u_pytest_jit.log"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$OUT/u_pytest_jit.log" | tail -25
echo "== A/B"
{
  AB_K=10 AB_M=8 timeout -k 10 300 python -u tools/ab.py "op=rec8,jit=0" "op=rec8,jit=2" "op=rec5,jit=0" "op=rec5,jit=2" "op=rec6,jit=0" "op=rec6,jit=2" "op=rec8p,jit=0" "op=rec8p,jit=2" "op=upd,jit=0" "op=upd,jit=2" "op=rep3,jit=0" "op=rep3,jit=2" &&
  AB_K=16 AB_M=8 timeout -k 10 300 python -u tools/ab.py "jit=0" "jit=2" "layout=inter,jit=0" "layout=inter,jit=2" &&
  AB_K=10 AB_M=8 timeout -k 10 300 python -u tools/ab.py "bitslice=1" "bitslice=0,jit=2" "bitslice=0,jit=0"
} > "$OUT/ab_jit.log" 2>&1 || { cat "$OUT/ab_jit.log" | tail -30; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit.log"
