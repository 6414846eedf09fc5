#!/usr/bin/env bash
# Same-box A/B of one synchronous 10+4 host call (AB_SIZES, default 8 KiB;
# AB_OPS host_latency's op mask) between the
# current library and another build of it (default tools/_build/r03lib:
# the round-3 tree built from its commit), alternating A B A B so box drift
# hits both.  Every call's result is checked by tools/host_latency.c.
# Output: gpurun_out/engine_ab.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OTHER="${1:-tools/_build/r03lib}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_latency.c -L"$OTHER" -lrsamd \
    -Wl,-rpath,"$PWD/$OTHER" -o tools/_build/host_latency_other
{
  for i in 1 2; do
    for v in host_latency host_latency_other; do
      echo "# $v pageable ($i)"; timeout -k 10 120 env HL_SIZES="${AB_SIZES:-8192}" HL_OPS="${AB_OPS:-31}" tools/_build/$v | grep '^{"op"'
      echo "# $v registered ($i)"; timeout -k 10 120 env HL_SIZES="${AB_SIZES:-8192}" HL_OPS="${AB_OPS:-31}" HL_REGISTER=1 tools/_build/$v | grep '^{"op"'
    done
  done
} > gpurun_out/engine_ab.log 2>&1
