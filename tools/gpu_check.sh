#!/usr/bin/env bash
# GPU-box check: smoke -> gpu tests -> bench (each step time-limited; stop at first failure).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
echo "== smoke"; timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -2 "$OUT/smoke.log"
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
echo "== bench"; timeout -k 10 400 python -u bench.py --cpu-seconds 10 > "$OUT/bench.log" 2>&1
cat "$OUT/bench.log"
