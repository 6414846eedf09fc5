#!/usr/bin/env bash
# Round-2 GPU pass d: full gpu suite (host-call engine on by default), host
# latency and concurrency with the engine on / off.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
echo "== engine tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_engine.log" 2>&1 || { tail -40 "$OUT/pytest_engine.log"; exit 1; }
tail -2 "$OUT/pytest_engine.log"
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
echo "== host latency"
{
  echo "# engine on (default, 8 workgroups)"; HL_ENGINE=1 timeout -k 10 200 tools/_build/host_latency
  echo "# engine on, 4 workgroups"; HL_ENGINE=1 HL_ENGINE_WAVES=4 timeout -k 10 200 tools/_build/host_latency
  echo "# engine on, 16 workgroups"; HL_ENGINE=1 HL_ENGINE_WAVES=16 timeout -k 10 200 tools/_build/host_latency
  echo "# engine off (launch + stream sync per call)"; HL_ENGINE=0 timeout -k 10 200 tools/_build/host_latency
} > "$OUT/host_latency_engine.log" 2>&1
grep -E '^#|"vec": (4096|8192|65536),' "$OUT/host_latency_engine.log" | grep -E '^#|Encode|lost=4|Update' 
echo "== host concurrency 8 KiB"
{
  echo "# engine on"; HL_ENGINE=1 timeout -k 10 200 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 32 64
  echo "# engine off"; HL_ENGINE=0 timeout -k 10 200 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 32 64
  echo "# engine on, mixed"; HL_ENGINE=1 timeout -k 10 200 tools/_build/host_concurrency 8192 300 131072 1 1 2 4 8 16 32 64
} > "$OUT/host_concurrency_engine.log" 2>&1
cat "$OUT/host_concurrency_engine.log" | cut -c1-200
