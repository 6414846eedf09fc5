#!/usr/bin/env bash
# Round-2 GPU pass m: the registered-memory concurrency hang (wg_units 64), traced.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
export RSAMD_TEARDOWN_TRACE=1 HL_PROGRESS=1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
echo "# registered, wg_units 0"
HL_REGISTER=1 timeout -k 5 40 tools/_build/host_concurrency 8192 300 131072 0 1 8 > "$OUT/m0.out" 2> "$OUT/m0.err" || { echo "rc $?"; tail -5 "$OUT/m0.err"; exit 1; }
cut -c1-150 "$OUT/m0.out"
echo "# registered, wg_units 64, traced"
RSAMD_ENGINE_TRACE=1 HL_ENGINE_WG_UNITS=64 HL_REGISTER=1 timeout -k 5 40 tools/_build/host_concurrency 8192 300 131072 0 1 8 > "$OUT/m1.out" 2> "$OUT/m1.err" || { echo "rc $?"; cut -c1-300 "$OUT/m1.out"; grep -v slow "$OUT/m1.err" | tail -30 | cut -c1-300; exit 1; }
cut -c1-150 "$OUT/m1.out"
