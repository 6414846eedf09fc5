#!/usr/bin/env bash
# Round-2 GPU pass w: full validation of the tree (smoke, every GPU test, the
# driver's bench command, its rocprof kernel trace, per-op table).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT/prof_w"
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/w_smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $OUT/w_smoke.log; exit 1; }
tail -1 $OUT/w_smoke.log
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/w_pytest_gpu.log 2>&1 || { echo "pytest rc $?"; tail -40 $OUT/w_pytest_gpu.log; exit 1; }
tail -1 $OUT/w_pytest_gpu.log
echo "== bench (driver command)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/w_bench.log 2>&1 || { echo "bench rc $?"; tail -20 $OUT/w_bench.log; exit 1; }
grep '^{' $OUT/w_bench.log | cut -c1-400
echo "== rocprof kernel trace of the driver command"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_w/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/prof_w/kt_bench.log" 2>&1 ) || { echo "rocprof rc $?"; tail -20 "$OUT/prof_w/kt_bench.log"; exit 1; }
grep '^{' "$OUT/prof_w/kt_bench.log" | cut -c1-300
echo "== ops bench"
timeout -k 10 600 python -u tools/ops_bench.py > $OUT/w_ops_bench.log 2>&1 || { echo "ops rc $?"; tail -30 $OUT/w_ops_bench.log; exit 1; }
grep -v amdgpu.ids $OUT/w_ops_bench.log
