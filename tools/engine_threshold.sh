#!/usr/bin/env bash
# Where the resident host-call engine stops paying: one call's latency
# (tools/host_latency.c, Encode, 8-64 KiB vectors, pageable and registered)
# and 1 / 8 concurrent callers' throughput (tools/host_concurrency.c) with
# the engine taking stripes up to the default 1 MiB and up to 14 x 16 / 32 KiB.
# Every call's result is checked.  Output: gpurun_out/engine_threshold.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
for t in host_latency host_concurrency; do
  gcc -O2 -std=c99 -pthread -Iinclude tools/$t.c -Lreedsolomon_amd/_lib -lrsamd \
      -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/$t
done
{
  for max in 1048576 229376 458752; do
    for reg in 0 1; do
      echo "# latency engine_max=$max registered=$reg"
      timeout -k 10 200 env HL_OPS=1 HL_SIZES=8192,16384,24576,32768,49152,65536 HL_ENGINE_MAX=$max HL_REGISTER=$reg \
          tools/_build/host_latency 2>&1 | grep '^{"op"'
    done
    for vec in 32768 65536; do
      echo "# concurrency engine_max=$max vec=$vec"
      timeout -k 10 200 env HL_ENGINE_MAX=$max tools/_build/host_concurrency $vec 200 131072 0 1 8 2>&1 | grep '^{"threads"'
    done
  done
} > gpurun_out/engine_threshold.log 2>&1
