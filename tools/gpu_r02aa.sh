#!/usr/bin/env bash
# Round-2 GPU pass aa: in-place Reconst on the interleaved layout, compiled vs perm-table kernels.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
{
  AB_K=10 AB_M=8 timeout -k 10 300 python -u tools/ab.py "op=rec8,layout=inter,jit=0" "op=rec8,layout=inter,jit=2" "op=rec8,jit=0" "op=rec8,jit=2" "op=rec5,layout=inter,jit=0" "op=rec5,layout=inter,jit=2" "layout=inter,bitslice=1" "bitslice=1" &&
  timeout -k 10 300 python -u tools/ab.py "op=rec4,layout=inter" "op=rec4" "op=rec2,layout=inter" "op=rec2"
} > "$OUT/ab_inter_rec.log" 2>&1 || { tail -30 "$OUT/ab_inter_rec.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_inter_rec.log"
