#!/usr/bin/env bash
# Round-2 GPU pass z: XCD-contiguous chunk remap A/B on the one-chunk kernels.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
{
  timeout -k 10 300 python -u tools/ab.py "xcd_remap=0" "xcd_remap=1" "layout=inter,xcd_remap=0" "layout=inter,xcd_remap=1" "op=rec4,xcd_remap=0" "op=rec4,xcd_remap=1" &&
  AB_VEC=8192 timeout -k 10 300 python -u tools/ab.py "xcd_remap=0" "xcd_remap=1" "op=upd,xcd_remap=0" "op=upd,xcd_remap=1" &&
  AB_K=12 timeout -k 10 300 python -u tools/ab.py "xcd_remap=0" "xcd_remap=1"
} > "$OUT/ab_xcd.log" 2>&1 || { tail -30 "$OUT/ab_xcd.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_xcd.log"
