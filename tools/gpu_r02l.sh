#!/usr/bin/env bash
# Round-2 GPU pass l: direct engine calls (no coalescing), engine geometry
# sweep (workgroups x waves, units per workgroup): latency and concurrency.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
export RSAMD_TEARDOWN_TRACE=1 RSAMD_WATCHDOG=1 HL_PROGRESS=1
echo "== engine + host-call tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "engine or host or coalesc or concurrent or staging or registered" > "$OUT/pytest_engine.log" 2>&1 || { tail -40 "$OUT/pytest_engine.log"; exit 1; }
tail -2 "$OUT/pytest_engine.log"
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
{
  for CFG in "8 8 64" "8 8 0" "16 2 64" "32 1 64" "32 2 64" "64 1 64" "16 4 128"; do
    set -- $CFG
    export HL_ENGINE_WAVES=$1 HL_ENGINE_GROUP_WAVES=$2 HL_ENGINE_WG_UNITS=$3
    echo "# groups $1 waves/group $2 units/group $3"
    HL_VEC=8192 HL_OPS=9 timeout -k 10 60 tools/_build/host_latency | grep -v engine_
    HL_REGISTER=1 HL_VEC=8192 HL_OPS=9 timeout -k 10 60 tools/_build/host_latency | grep -v engine_ | sed 's/^/reg /'
    timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64 | grep -v engine_
    HL_REGISTER=1 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 8 | grep -v engine_ | sed 's/^/reg /'
  done
  unset HL_ENGINE_WAVES HL_ENGINE_GROUP_WAVES HL_ENGINE_WG_UNITS
  echo "# coalescing (direct off), defaults"
  HL_ENGINE_DIRECT=0 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16 64 | grep -v engine_
  echo "# defaults, mixed"
  timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 1 1 2 8 64 | grep -v engine_
} > "$OUT/engine_l.log" 2>&1
cut -c1-150 "$OUT/engine_l.log"
