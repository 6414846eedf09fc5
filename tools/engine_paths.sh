#!/usr/bin/env bash
# The resident host-call engine's small-call figures in one pass: one 10+4
# @ 8 KiB call's latency from pageable and from registered memory
# (tools/host_latency.c) and T concurrent callers' throughput
# (tools/host_concurrency.c).  Every call's result is checked by the tools.
# Output: gpurun_out/engine_paths.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
for t in host_latency host_concurrency; do
  gcc -O2 -std=c99 -pthread -Iinclude tools/$t.c -Lreedsolomon_amd/_lib -lrsamd \
      -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/$t
done
run() { echo "# $1"; shift; timeout -k 10 200 "$@"; }
{
  run "one call, pageable vectors" env HL_VEC=8192 tools/_build/host_latency
  run "one call, registered vectors" env HL_VEC=8192 HL_REGISTER=1 tools/_build/host_latency
  run "T threads, 8 KiB Encode, pageable" tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16
  run "T threads, 8 KiB Encode, registered" env HL_REGISTER=1 tools/_build/host_concurrency 8192 300 131072 0 1 2 4 8 16
} > gpurun_out/engine_paths.log 2>&1
