#!/usr/bin/env bash
# Round-2 GPU pass o: host_concurrency exit hang: kernel-side state of the
# hung process's threads (/proc wchan / syscall), then kill it.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
export RSAMD_TEARDOWN_TRACE=1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency || exit 1
for R in $(seq 1 24); do
  HL_ENGINE_WAVES=16 HL_ENGINE_GROUP_WAVES=2 HL_ENGINE_WG_UNITS=64 HL_REGISTER=${REG:-1} \
      tools/_build/host_concurrency 8192 300 131072 0 1 8 > "$OUT/o$R.out" 2> "$OUT/o$R.err" &
  pid=$!
  for i in $(seq 1 80); do
    kill -0 $pid 2>/dev/null || break
    sleep 0.1
  done
  if kill -0 $pid 2>/dev/null; then
    echo "run $R: pid $pid still alive after 8 s; stderr tail: $(tail -2 "$OUT/o$R.err" | tr '\n' '|')"
    for t in /proc/$pid/task/*; do
      echo "  task $(basename $t) $(cat $t/comm 2>/dev/null) wchan=$(cat $t/wchan 2>/dev/null) state=$(awk '{print $3}' $t/stat 2>/dev/null) syscall=$(cat $t/syscall 2>/dev/null | cut -d' ' -f1-3)"
      cat $t/stack 2>/dev/null | head -12 | sed 's/^/      /'
    done
    cat /proc/$pid/status | grep -E "State|Threads"
    kill -9 $pid; wait $pid 2>/dev/null
    exit 9
  fi
  wait $pid; echo "run $R rc $?"
done
