#!/usr/bin/env bash
# Round-2 GPU pass t: adaptive engine spreading (lone calls over every
# workgroup); latency with the phase trace, thread sweep, engine tests.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency || exit 1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
HL=tools/_build/host_latency; HC=tools/_build/host_concurrency
step() { echo "# $1"; shift; timeout -k 10 120 "$@" 2>&1 | grep -v '^host_\|^{"engine' || { echo "step rc $?"; exit 1; }; }
{
  step "pageable latency" env HL_VEC=8192 $HL
  step "registered latency" env HL_REGISTER=1 HL_VEC=8192 $HL
  step "pageable latency, phase trace (Encode)" env RSAMD_ENGINE_TRACE=1 HL_VEC=8192 HL_OPS=1 $HL
  step "registered latency, phase trace (Encode)" env RSAMD_ENGINE_TRACE=1 HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 $HL
  step "pageable threads" $HC 8192 300 131072 0 1 2 4 8 16 64
  step "registered threads" env HL_REGISTER=1 $HC 8192 300 131072 0 1 2 4 8 16
  step "pageable threads, mixed" $HC 8192 300 131072 1 1 2 8 16
  step "64 KiB latency" env HL_VEC=65536 HL_OPS=1 $HL
  step "64 KiB threads" $HC 65536 200 131072 0 1 2 8 16
} > "$OUT/engine_t.log" 2>&1 || { cat "$OUT/engine_t.log" | cut -c1-200; exit 1; }
cut -c1-200 "$OUT/engine_t.log"
echo "== engine tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/t_pytest_engine.log" 2>&1 || { tail -30 "$OUT/t_pytest_engine.log"; exit 1; }
tail -1 "$OUT/t_pytest_engine.log"
