#!/usr/bin/env bash
# Diagnostic: the gpu suite with the host-call engine off (RSAMD_HOST_ENGINE=0).
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
echo "== pytest -m gpu, engine off"
RSAMD_HOST_ENGINE=0 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider --deselect tests/test_gpu_engine.py > "$OUT/pytest_gpu_noengine.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_noengine.log"; exit 1; }
tail -2 "$OUT/pytest_gpu_noengine.log"
