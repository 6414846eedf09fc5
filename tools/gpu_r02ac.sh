#!/usr/bin/env bash
# Round-2 GPU pass ac: JIT recurrence policy (tests), then the concurrency stress.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/ac_pytest.log" 2>&1 || { tail -60 "$OUT/ac_pytest.log"; exit 1; }
tail -1 "$OUT/ac_pytest.log"
timeout -k 10 240 python -u tools/gpu_stress.py 8 75 > "$OUT/stress_ac.log" 2>&1 || { echo "stress rc $?"; tail -20 "$OUT/stress_ac.log"; exit 1; }
tail -1 "$OUT/stress_ac.log"
