#!/usr/bin/env bash
# Round-2 GPU pass f: engine tests (coherent pool buffers, fence-free), host
# latency and concurrency with the engine's batch limit swept.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
echo "== engine + host-call tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "engine or host or coalesc or concurrent or staging" > "$OUT/pytest_engine.log" 2>&1 || { tail -40 "$OUT/pytest_engine.log"; exit 1; }
tail -2 "$OUT/pytest_engine.log"
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
echo "== host latency"
{
  echo "# engine on (8 workgroups, coherent pool buffers, no fences)"; HL_ENGINE=1 timeout -k 10 200 tools/_build/host_latency
  echo "# engine off"; HL_ENGINE=0 timeout -k 10 200 tools/_build/host_latency
} > "$OUT/host_latency_engine2.log" 2>&1
grep -E '^#|"vec": (4096|8192|65536),|engine' "$OUT/host_latency_engine2.log" | grep -E '^#|Encode|lost=4|Update|engine'
echo "== host concurrency 8 KiB"
{
  for M in 1048576 262144 131072; do
    echo "# engine on, max $M"; HL_ENGINE=1 HL_ENGINE_MAX=$M timeout -k 10 200 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  done
  echo "# engine off"; HL_ENGINE=0 timeout -k 10 200 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  echo "# engine on, max 262144, 64 KiB"; HL_ENGINE=1 HL_ENGINE_MAX=262144 timeout -k 10 200 tools/_build/host_concurrency 65536 200 131072 0 1 2 8 64
  echo "# engine off, 64 KiB"; HL_ENGINE=0 timeout -k 10 200 tools/_build/host_concurrency 65536 200 131072 0 1 2 8 64
} > "$OUT/host_concurrency_engine2.log" 2>&1
cut -c1-175 "$OUT/host_concurrency_engine2.log"
