#!/usr/bin/env bash
# Engine workgroups 8 vs 16 for 1 / 8 / 16 concurrent 8 KiB host Encode callers (tools/host_concurrency.c). Output: gpurun_out/engine_wg16.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
{
for i in 1 2; do
  for wg in 8 16; do
    echo "# wg=$wg pageable ($i)"; timeout -k 10 200 env HL_ENGINE_WAVES=$wg tools/_build/host_concurrency 8192 300 131072 0 1 8 16 2>&1 | grep '^{"threads"'
  done
done
} > gpurun_out/engine_wg16.log 2>&1
