#!/usr/bin/env bash
# Round-2 GPU pass am: pipelined doorbell polls (host_engine_poll_gap): engine
# tests with the gap on, then latency / concurrency A/B over gaps.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency || exit 1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
HL=tools/_build/host_latency; HC=tools/_build/host_concurrency
RSAMD_ENGINE_POLL_GAP=100 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/am_pytest_engine.log" 2>&1 || { tail -40 "$OUT/am_pytest_engine.log"; exit 1; }
tail -1 "$OUT/am_pytest_engine.log"
step() { echo "# $1"; shift; timeout -k 10 120 "$@" 2>&1 | grep -v '^host_\|^{"engine' || { echo "step rc $?"; exit 1; }; }
{
  step "gap 100: pageable latency (check run)" env HL_ENGINE_POLL_GAP=100 HL_VEC=8192 HL_OPS=1 $HL
  for R in 1 2; do
    for G in 0 50 100 150; do
      step "gap $G run $R: pageable" env HL_ENGINE_POLL_GAP=$G HL_VEC=8192 $HL
      step "gap $G run $R: registered" env HL_ENGINE_POLL_GAP=$G HL_REGISTER=1 HL_VEC=8192 HL_OPS=9 $HL
    done
  done
  for G in 0 100; do step "gap $G: threads" env HL_ENGINE_POLL_GAP=$G $HC 8192 300 131072 0 1 2 8 16; done
} > "$OUT/engine_am.log" 2>&1 || { cut -c1-160 "$OUT/engine_am.log"; exit 1; }
cut -c1-140 "$OUT/engine_am.log"
