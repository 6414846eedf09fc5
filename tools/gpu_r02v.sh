#!/usr/bin/env bash
# Round-2 GPU pass v: JIT tests after the accumulate rule; prefetch distance
# and workgroup size of the compiled kernels (16+8 Encode, 10+8 Reconst of 8).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/v_pytest_jit.log" 2>&1 || { tail -60 "$OUT/v_pytest_jit.log"; exit 1; }
tail -1 "$OUT/v_pytest_jit.log"
{
  AB_K=16 AB_M=8 timeout -k 10 300 python -u tools/ab.py "jit_pf=2" "jit_pf=3" "jit_pf=4" "jit_pf=5" "bs_block=256" "bs_block=256,jit_pf=4" &&
  AB_K=10 AB_M=8 timeout -k 10 300 python -u tools/ab.py "op=rec8,jit_pf=2" "op=rec8,jit_pf=3" "op=rec8,jit_pf=4" "op=rec8,bs_block=256"
} > "$OUT/ab_jit_pf.log" 2>&1 || { tail -30 "$OUT/ab_jit_pf.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_pf.log"
