#!/usr/bin/env bash
# Host-call latency sweep on the GPU box (tools/host_latency.c): staging
# paths, chunk sizes and copy-thread counts.  Output: gpurun_out/host_latency.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
run() { echo "# $1"; shift; timeout -k 10 200 "$@"; }
{
  run "default (chunked zero-copy, 256 KiB chunks, 4 copy threads)" tools/_build/host_latency
  run "chunk 128 KiB" tools/_build/host_latency -1 262144 131072
  run "chunk 1 MiB" tools/_build/host_latency -1 262144 1048576
  run "1 copy thread" env RSAMD_HOST_THREADS=1 tools/_build/host_latency
  run "8 copy threads" env RSAMD_HOST_THREADS=8 tools/_build/host_latency
  run "registered caller vectors (rs_host_register): zero-copy over them" env HL_REGISTER=1 tools/_build/host_latency
  run "staged: pinned mirror + DMA <= 4 MiB" tools/_build/host_latency 0 4194304
  run "staged: pageable per-vector copies" tools/_build/host_latency 0 0
} > gpurun_out/host_latency.log 2>&1
