#!/usr/bin/env bash
# Round-2 GPU pass j: find the host_concurrency exit hang (engine traces).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
for R in 1 2 3; do
  echo "# run $R"
  RSAMD_ENGINE_TRACE=1 timeout -k 5 40 tools/_build/host_concurrency 8192 300 131072 0 1 8 16 64 > "$OUT/hang_$R.out" 2> "$OUT/hang_$R.err"
  rc=$?
  echo "rc $rc"; cut -c1-160 "$OUT/hang_$R.out"; grep -v "slow" "$OUT/hang_$R.err" | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
