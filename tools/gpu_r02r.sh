#!/usr/bin/env bash
# Round-2 GPU pass r: the reworked host-call engine (call slots, direct calls)
# against engine off: 10+4 host-call latency (pageable / registered) and
# concurrent throughput, 8 KiB and 64 KiB.  Output: gpurun_out/engine_r.log
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency || exit 1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
HL=tools/_build/host_latency; HC=tools/_build/host_concurrency
step() { echo "# $1"; shift; timeout -k 10 120 "$@" || { echo "step rc $?"; exit 1; }; }
{
  for E in 1 0; do
    step "engine $E, pageable, latency" env HL_ENGINE=$E HL_VEC=8192 $HL
    step "engine $E, registered, latency" env HL_ENGINE=$E HL_REGISTER=1 HL_VEC=8192 $HL
    step "engine $E, pageable, 64 KiB latency" env HL_ENGINE=$E HL_VEC=65536 HL_OPS=1 $HL
    step "engine $E, pageable, 8 KiB threads" env HL_ENGINE=$E $HC 8192 300 131072 0 1 2 4 8 16 64
    step "engine $E, registered, 8 KiB threads" env HL_ENGINE=$E HL_REGISTER=1 $HC 8192 300 131072 0 1 2 4 8 16
    step "engine $E, pageable, 8 KiB threads, mixed" env HL_ENGINE=$E $HC 8192 300 131072 1 1 2 8 16
    step "engine $E, pageable, 64 KiB threads" env HL_ENGINE=$E $HC 65536 200 131072 0 1 2 8 16
  done
} > "$OUT/engine_r.log" 2>&1
rc=$?
grep -v '^{"engine' "$OUT/engine_r.log" | cut -c1-200
exit $rc
