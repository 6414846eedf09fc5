#!/usr/bin/env bash
# Round-2 GPU pass ah: run-time kernels up to 16 rows (tests, A/B vs the
# perm-table row groups), then the ops table refresh.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_jit.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/ah_pytest_jit.log" 2>&1 || { tail -60 "$OUT/ah_pytest_jit.log"; exit 1; }
tail -1 "$OUT/ah_pytest_jit.log"
{
  AB_K=20 AB_M=12 timeout -k 10 300 python -u tools/ab.py "op=rec12,jit=0" "op=rec12,jit=2" "jit=0" "jit=2" &&
  AB_K=16 AB_M=16 timeout -k 10 300 python -u tools/ab.py "op=rec16,jit=0" "op=rec16,jit=2" "jit=0" "jit=2"
} > "$OUT/ab_jit16.log" 2>&1 || { tail -30 "$OUT/ab_jit16.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit16.log"
timeout -k 10 600 python -u tools/ops_bench.py > $OUT/ag_ops_bench.log 2>&1 || { echo "ops rc $?"; tail -30 $OUT/ag_ops_bench.log; exit 1; }
grep -v amdgpu.ids $OUT/ag_ops_bench.log | head -36
