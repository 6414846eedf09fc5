#!/usr/bin/env bash
# Round-2 GPU pass y: engine waiters yield after 30 us (oversubscribed callers),
# JIT worker lifetime rework: engine + JIT tests, thread sweep with / without yield.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_jit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/y_pytest.log" 2>&1 || { tail -60 "$OUT/y_pytest.log"; exit 1; }
tail -1 "$OUT/y_pytest.log"
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
HC=tools/_build/host_concurrency
step() { echo "# $1"; shift; timeout -k 10 120 "$@" 2>&1 | grep -v '^host_\|^{"engine' || { echo "step rc $?"; exit 1; }; }
{
  for R in 1 2; do
    step "yield after 30 us (default), run $R" $HC 8192 300 131072 0 1 2 4 8 16 32 64
    step "never yield, run $R" env HL_ENGINE_YIELD=0 $HC 8192 300 131072 0 1 2 4 8 16 32 64
  done
  step "yield, 64 KiB" $HC 65536 200 131072 0 1 2 8 16 64
  step "yield, mixed" $HC 8192 300 131072 1 1 2 8 16 64
} > "$OUT/engine_y.log" 2>&1 || { cat "$OUT/engine_y.log" | cut -c1-200; exit 1; }
cut -c1-170 "$OUT/engine_y.log"
