#!/usr/bin/env bash
# Host-call engine sweep: workgroups x batch limit, 8 KiB calls, T threads.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"; mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
{
for cfg in "8 131072" "16 524288" "32 1048576" "64 2097152"; do
  set -- $cfg
  echo "# waves $1 max $2"
  HL_ENGINE=1 HL_ENGINE_WAVES=$1 HL_ENGINE_MAX=$2 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 8 16 64 | grep threads
  HL_ENGINE=1 HL_ENGINE_WAVES=$1 HL_ENGINE_MAX=$2 timeout -k 10 100 tools/_build/host_latency | grep -E '"vec": 8192' | head -3
done
} > gpurun_out/engine_sweep.log 2>&1
cut -c1-160 gpurun_out/engine_sweep.log
