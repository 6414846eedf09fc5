#!/usr/bin/env bash
# Round-2 GPU pass ad: process exit while the JIT worker compiles (the SIGSEGV
# at exit of pass ac): stress twice with compiles in flight at exit, once with JIT off.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
cd "$OUT"   # (a core file, if any, stays out of the repo root)
ulimit -c 0
for R in 1 2; do
  timeout -k 10 200 python -u "$REPO/tools/gpu_stress.py" 8 40 > "$OUT/stress_ad_$R.log" 2>&1; rc=$?
  echo "run $R rc $rc: $(tail -1 "$OUT/stress_ad_$R.log" | cut -c1-220)"
  [ $rc -eq 0 ] || exit 1
done
RSAMD_JIT=0 timeout -k 10 200 python -u "$REPO/tools/gpu_stress.py" 8 30 > "$OUT/stress_ad_nojit.log" 2>&1; rc=$?
echo "jit off rc $rc: $(tail -1 "$OUT/stress_ad_nojit.log" | cut -c1-220)"
exit $rc
