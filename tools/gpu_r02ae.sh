#!/usr/bin/env bash
# Round-2 GPU pass ae: exit during the FIRST background compile, 5 processes.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"; cd "$OUT"; ulimit -c 0
for R in 1 2 3 4 5; do
  s=$(date +%s.%N)
  timeout -k 10 90 python -u "$REPO/tools/jit_exit_probe.py" $R > "$OUT/exit_probe_$R.log" 2>&1; rc=$?
  e=$(date +%s.%N)
  echo "run $R rc $rc $(python3 -c "print(round($e-$s,1))") s: $(grep -v amdgpu.ids "$OUT/exit_probe_$R.log" | tail -1 | cut -c1-120)"
  [ $rc -eq 0 ] || exit 1
done
