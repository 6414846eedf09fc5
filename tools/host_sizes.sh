#!/usr/bin/env bash
# One synchronous 10+4 host-memory Encode across vector sizes (4 KiB - 4 MiB),
# per host path: the default (resident engine up to host_engine_max_bytes,
# then the chunked zero-copy pipeline, staged above host_zc_max), the engine
# off, the engine capped at 256 KiB, and registered memory; plus the engine's
# phase trace at 1 MiB.  Every call's result is checked by tools/host_latency.c.
# Output: gpurun_out/host_sizes.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
run() { echo "# $1"; shift; timeout -k 10 200 env HL_OPS=1 "$@" tools/_build/host_latency 2>&1 | grep -v '^host_latency:'; }
{
  run "default (pageable)"
  run "engine off (pageable)" HL_ENGINE=0
  run "engine up to 256 KiB (pageable)" HL_ENGINE_MAX=262144
  run "registered" HL_REGISTER=1
  run "default, 1 MiB, engine phase trace" HL_VEC=1048576 RSAMD_ENGINE_TRACE=1
} > gpurun_out/host_sizes.log 2>&1
