#!/usr/bin/env bash
# Round-2 GPU pass s: engine geometry vs single-call latency (10+4 @ 8 KiB, pageable and registered)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency || exit 1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
HL=tools/_build/host_latency; HC=tools/_build/host_concurrency
step() { echo "# $1"; shift; timeout -k 10 120 "$@" 2>&1 | grep -v '^host_\|^{"engine' || { echo "step rc $?"; exit 1; }; }
{
  for CFG in "8 8 0" "8 8 64" "8 8 128" "16 4 64" "32 2 32" "32 1 16" "64 1 16" "16 2 32"; do
    set -- $CFG
    export HL_ENGINE_WAVES=$1 HL_ENGINE_GROUP_WAVES=$2 HL_ENGINE_WG_UNITS=$3
    step "groups $1 waves/group $2 units/wg $3: pageable" env HL_VEC=8192 HL_OPS=7 $HL
    step "groups $1 waves/group $2 units/wg $3: registered" env HL_REGISTER=1 HL_VEC=8192 HL_OPS=7 $HL
    step "groups $1 waves/group $2 units/wg $3: threads" $HC 8192 300 131072 0 1 2 8 16
  done
} > "$OUT/engine_s.log" 2>&1
cat "$OUT/engine_s.log" | cut -c1-170
