#!/usr/bin/env bash
# Concurrent host-call throughput with and without coalescing
# (tools/host_concurrency.c).  Output: gpurun_out/host_concurrency.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
B=tools/_build/host_concurrency
{
  for V in 8192 65536; do
    for MIX in 0 1; do
      echo "# vec $V mixed $MIX: coalescing on (default 128 KiB)"
      timeout -k 10 120 $B $V 300 131072 $MIX 1 2 4 8 16 32 64
      echo "# vec $V mixed $MIX: coalescing off"
      timeout -k 10 120 $B $V 300 0 $MIX 1 2 4 8 16 32 64
    done
  done
} > gpurun_out/host_concurrency.log 2>&1
