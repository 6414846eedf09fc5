#!/usr/bin/env bash
# Round-2 GPU pass ap: compiled XOR-accumulate kernels with the old outputs
# loaded up front: JIT tests, then Update / Replace A/B at 10+8 and 16+8.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/ap_pytest_jit.log" 2>&1 || { tail -60 "$OUT/ap_pytest_jit.log"; exit 1; }
tail -1 "$OUT/ap_pytest_jit.log"
{
  AB_K=10 AB_M=8 timeout -k 10 400 python -u tools/ab.py "op=upd" "op=upd,jit_min_acc_cols=1" "op=rep3" "op=rep3,jit_min_acc_cols=1" &&
  AB_K=16 AB_M=8 timeout -k 10 400 python -u tools/ab.py "op=upd" "op=upd,jit_min_acc_cols=1" "op=rep3" "op=rep3,jit_min_acc_cols=1"
} > "$OUT/ab_jit_acc.log" 2>&1 || { tail -30 "$OUT/ab_jit_acc.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_acc.log"
