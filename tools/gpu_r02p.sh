#!/usr/bin/env bash
# Round-2 GPU pass p: exit hang A/B: the library before the engine rework
# (tools/_old, commit d2c7c1b) vs now, pageable 8 KiB concurrency, repeated.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT" tools/_build
gcc -O2 -std=c99 -pthread -Itools/_old tools/_old/host_concurrency_old.c -Ltools/_old -lrsamd \
    -Wl,-rpath,"$PWD/tools/_old" -o tools/_build/host_concurrency_old || exit 1
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -rdynamic -o tools/_build/host_concurrency || exit 1
run_loop() {  # name binary n
  for R in $(seq 1 $3); do
    $2 8192 100 131072 0 1 8 > "$OUT/p_$1_$R.out" 2> "$OUT/p_$1_$R.err" &
    pid=$!
    for i in $(seq 1 100); do kill -0 $pid 2>/dev/null || break; sleep 0.1; done
    if kill -0 $pid 2>/dev/null; then
      echo "$1 run $R: still alive after 10 s: $(tail -1 "$OUT/p_$1_$R.out" | cut -c1-80)"
      for t in /proc/$pid/task/*; do echo "  $(cat $t/comm) wchan=$(cat $t/wchan)"; done
      for t in /proc/$pid/task/*; do
        python3 -c "import ctypes,sys; ctypes.CDLL(None).syscall(234, int(sys.argv[1]), int(sys.argv[2]), 10)" $pid $(basename $t)
        sleep 0.5
      done
      sleep 1
      grep -A30 "thread stack" "$OUT/p_$1_$R.err" | grep -v "libc.so.6(+0x42520)\|host_concurrency(+0x" | head -100
      cat /proc/$pid/maps | grep -E "r-xp" | awk '{print $1, $6}' | grep -E "amdhip|hsa|rsamd|libc" | head -12
      kill -9 $pid; wait $pid 2>/dev/null
      return 9
    fi
    wait $pid || { echo "$1 run $R rc $?"; return 1; }
  done
  echo "$1: $3 runs exited cleanly"
}
if [ -n "${OLD:-}" ]; then run_loop old tools/_build/host_concurrency_old ${N:-20} || exit $?; fi
run_loop new${VARIANT:+_$VARIANT} tools/_build/host_concurrency ${N:-20} || exit $?
