#!/usr/bin/env bash
# Round-2 GPU pass g: where the time of a small synchronous host call goes
# (RSAMD_ENGINE_TRACE phase means, engine workgroup 0's GPU stamps).
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
{
  for OPS in 1 2 8; do
    echo "# engine on, 8 KiB, ops $OPS, traced"
    RSAMD_ENGINE_TRACE=1 HL_VEC=8192 HL_OPS=$OPS timeout -k 10 60 tools/_build/host_latency 2>&1 | grep -v "slow"
  done
  echo "# engine on, 8 KiB Encode, untraced"; HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency
  echo "# registered memory (launch path), 8 KiB Encode"; HL_REGISTER=1 HL_VEC=8192 HL_OPS=1 timeout -k 10 60 tools/_build/host_latency
  echo "# T=8, traced"
  RSAMD_ENGINE_TRACE=1 timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 8 2>&1 | grep -v "slow"
} > "$OUT/host_phases.log" 2>&1
cat "$OUT/host_phases.log"
