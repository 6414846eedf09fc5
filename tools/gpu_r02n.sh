#!/usr/bin/env bash
# Round-2 GPU pass n: where does host_concurrency hang at exit?
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
export RSAMD_TEARDOWN_TRACE=1 RSAMD_WATCHDOG=1 HL_PROGRESS=1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
for R in 1 2 3 4 5 6 7 8; do
  t0=$(date +%s.%N)
  HL_ENGINE_WAVES=16 HL_ENGINE_GROUP_WAVES=2 HL_ENGINE_WG_UNITS=64 HL_FAST_EXIT=${FAST:-0} HL_REGISTER=${REG:-1} timeout -k 5 45 tools/_build/host_concurrency 8192 300 131072 0 1 8 > "$OUT/n$R.out" 2> "$OUT/n$R.err"
  rc=$?
  t1=$(date +%s.%N)
  echo "run $R rc $rc wall $(python3 -c "print(round($t1-$t0,2))") s: $(grep -c threads "$OUT/n$R.out") result lines; stderr tail: $(tail -2 "$OUT/n$R.err" | tr '\n' '|')"
  if [ $rc -ne 0 ]; then cat "$OUT/n$R.err" | grep -v "workers ready" | tail -20; exit $rc; fi
done
