#!/usr/bin/env bash
# Round-2 GPU pass k: engine slots (4 calls in flight, lock-free waiting),
# two coalesced batches in flight: tests, latency, concurrency A/B.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
echo "== engine + host-call tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "engine or host or coalesc or concurrent or staging or registered" > "$OUT/pytest_engine.log" 2>&1 || { tail -40 "$OUT/pytest_engine.log"; exit 1; }
tail -2 "$OUT/pytest_engine.log"
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
{
  echo "# pageable"; HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  echo "# registered"; HL_REGISTER=1 HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  echo "# registered, wg_units 64"; HL_ENGINE_WG_UNITS=64 HL_REGISTER=1 HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  echo "# pageable, wg_units 64"; HL_ENGINE_WG_UNITS=64 HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  for R in 1 2; do
    echo "# coalesced, 2 batches in flight, run $R"; timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
    echo "# coalesced, calls spread over all workgroups (wg_units 64), run $R"; HL_ENGINE_WG_UNITS=64 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  done
  echo "# coalesced, idle 1000 us"; HL_ENGINE_IDLE=1000 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  echo "# registered"; HL_REGISTER=1 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  echo "# registered, 16 groups"; HL_ENGINE_WAVES=16 HL_REGISTER=1 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  echo "# coalesced, mixed"; timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 1 1 2 8 64
} > "$OUT/engine_k.log" 2>&1
grep -v engine_calls "$OUT/engine_k.log" | cut -c1-175
