#!/usr/bin/env bash
# Round-2 GPU pass aq: compiled kernels for 3-4 output rows over many columns (jit_min_rows).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
{
  AB_K=16 AB_M=4 timeout -k 10 400 python -u tools/ab.py "jit_min_rows=5" "jit_min_rows=1" "layout=inter,jit_min_rows=5" "layout=inter,jit_min_rows=1" "op=rec4,jit_min_rows=5" "op=rec4,jit_min_rows=1" &&
  AB_K=24 AB_M=4 timeout -k 10 400 python -u tools/ab.py "jit_min_rows=5" "jit_min_rows=1" "op=rec4,jit_min_rows=5" "op=rec4,jit_min_rows=1" &&
  AB_K=10 AB_M=4 timeout -k 10 400 python -u tools/ab.py "jit_min_rows=5" "op=rec4,jit_min_rows=5" "op=rec4,jit_min_rows=1" "op=rec2,jit_min_rows=5" "op=rec2,jit_min_rows=1"
} > "$OUT/ab_jit_rows34.log" 2>&1 || { tail -30 "$OUT/ab_jit_rows34.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_jit_rows34.log"
