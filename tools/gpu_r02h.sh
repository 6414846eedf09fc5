#!/usr/bin/env bash
# Round-2 GPU pass h: engine with multi-wave workgroups (wave 0 polls):
# engine tests, 8 KiB latency, and a (workgroups, waves per workgroup,
# batch limit) sweep of 8 KiB host-call concurrency.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
echo "== engine tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_engine.log" 2>&1 || { tail -40 "$OUT/pytest_engine.log"; exit 1; }
tail -2 "$OUT/pytest_engine.log"
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
{
  for CFG in "8 8 1048576" "8 1 131072" "8 4 1048576" "16 4 1048576" "4 8 1048576" "8 8 4194304"; do
    set -- $CFG
    echo "# groups $1 group_waves $2 max $3"
    HL_ENGINE_WAVES=$1 HL_ENGINE_GROUP_WAVES=$2 HL_ENGINE_MAX=$3 HL_VEC=8192 timeout -k 10 60 tools/_build/host_latency
    HL_ENGINE_WAVES=$1 HL_ENGINE_GROUP_WAVES=$2 HL_ENGINE_MAX=$3 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64
  done
  echo "# defaults, traced, T=8"
  RSAMD_ENGINE_TRACE=1 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 8 2>&1 | grep -v slow
} > "$OUT/engine_groups_sweep.log" 2>&1
cut -c1-200 "$OUT/engine_groups_sweep.log"
