#!/usr/bin/env bash
# Round-2 GPU pass ab: JIT tests incl. 4 threads in background mode.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/ab_pytest_jit.log" 2>&1 || { tail -60 "$OUT/ab_pytest_jit.log"; exit 1; }
grep -E "concurrent|passed|failed" "$OUT/ab_pytest_jit.log" | tail -3
