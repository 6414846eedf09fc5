#!/usr/bin/env bash
# Round-2 GPU pass ag: ops table refresh (split-layout > 4-output rows, multi-pattern after the grouping fix).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -u tools/ops_bench.py > $OUT/ag_ops_bench.log 2>&1 || { echo "ops rc $?"; tail -30 $OUT/ag_ops_bench.log; exit 1; }
grep -v amdgpu.ids $OUT/ag_ops_bench.log | head -40
