#!/usr/bin/env bash
# Round-2 GPU pass i: engine epochs / gone words / address mode: engine and
# host-call tests, 8 KiB latency (pageable and registered), concurrency.
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
  echo "# pageable, defaults"; HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  echo "# registered, defaults"; HL_REGISTER=1 HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
  echo "# registered, traced"; RSAMD_ENGINE_TRACE=1 HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency 2>&1 | grep -v slow
  echo "# registered, group_waves 1"; HL_ENGINE_GROUP_WAVES=1 HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency
  echo "# registered, 4 groups"; HL_ENGINE_WAVES=4 HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency
  echo "# registered, 16 groups"; HL_ENGINE_WAVES=16 HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency
  for R in 1 2; do
    echo "# concurrency, defaults, run $R"; timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  done
  echo "# concurrency, group_waves 4"; HL_ENGINE_GROUP_WAVES=4 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
} > "$OUT/engine_i.log" 2>&1
cut -c1-200 "$OUT/engine_i.log"
