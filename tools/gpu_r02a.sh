#!/usr/bin/env bash
# Round-2 GPU check: gpu tests, the driver's exact bench command, the same
# command under rocprofv3 --kernel-trace --stats, smoke.  Each step has its
# own time limit; the script stops at the first failure.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "== driver bench command"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || { tail -20 "$OUT/bench_driver.log"; exit 1; }
grep '^{' "$OUT/bench_driver.log" | cut -c1-1500
echo "== driver bench command under rocprofv3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_prof.log" 2>&1 || { tail -20 "$OUT/bench_driver_prof.log"; exit 1; }
grep '^{' "$OUT/bench_driver_prof.log" | cut -c1-1500
cd "$REPO"
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
