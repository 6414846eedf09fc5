#!/usr/bin/env bash
# Round-2 GPU pass ao: 256-lane compiled kernels from 20 columns (tests + A/B check).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/ao_pytest_jit.log" 2>&1 || { tail -60 "$OUT/ao_pytest_jit.log"; exit 1; }
tail -1 "$OUT/ao_pytest_jit.log"
{
  AB_K=40 AB_M=8 AB_VEC=262144 timeout -k 10 400 python -u tools/ab.py "op=rec8" "op=rec8,jit=0" "jit=2" "jit=0" &&
  AB_K=20 AB_M=12 timeout -k 10 400 python -u tools/ab.py "op=rec12" "op=rec12,bs_block=64" &&
  AB_K=16 AB_M=8 timeout -k 10 400 python -u tools/ab.py "jit=2" "bs_block=256"
} > "$OUT/ab_jit_ao.log" 2>&1 || { tail -30 "$OUT/ab_jit_ao.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_ao.log"
