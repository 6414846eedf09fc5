#!/usr/bin/env bash
# Round-2 GPU pass x: multi-pattern host grouping fix (tests + A/B), JIT
# workgroup size on the interleaved layout.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "multi" > "$OUT/x_pytest_multi.log" 2>&1 || { tail -60 "$OUT/x_pytest_multi.log"; exit 1; }
tail -1 "$OUT/x_pytest_multi.log"
{
  AB_VEC=8192 timeout -k 10 300 python -u tools/ab.py "op=multi16" "op=multi16s" "op=rec4" "op=multi16,layout=inter" &&
  timeout -k 10 300 python -u tools/multi_mix.py &&
  AB_K=10 AB_M=8 timeout -k 10 300 python -u tools/ab.py "op=rec8,layout=inter" "op=rec8,layout=inter,bs_block=64" "op=rec5,layout=inter" "op=rec5,layout=inter,bs_block=64" "op=rec8" &&
  AB_K=16 AB_M=8 timeout -k 10 300 python -u tools/ab.py "layout=inter" "layout=inter,bs_block=64" "layout=inter,bs_block=128"
} > "$OUT/ab_x.log" 2>&1 || { tail -30 "$OUT/ab_x.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_x.log"
