#!/usr/bin/env bash
# Round-2 GPU pass al: the other bench configurations (12+4 @ 1 MiB, interleaved layout).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --config 12+4@1MiB --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/al_bench_12_4.log 2>&1 || { echo "rc $?"; tail -20 $OUT/al_bench_12_4.log; exit 1; }
grep '^{' $OUT/al_bench_12_4.log | cut -c1-260
timeout -k 10 300 python -u bench.py --layout interleaved --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/al_bench_inter.log 2>&1 || { echo "rc $?"; tail -20 $OUT/al_bench_inter.log; exit 1; }
grep '^{' $OUT/al_bench_inter.log | cut -c1-260
