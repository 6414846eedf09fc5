#!/usr/bin/env bash
# Round-2 GPU pass q: full check of the restored tree (smoke, every GPU test, the driver's bench command).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/q_smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $OUT/q_smoke.log; exit 1; }
tail -1 $OUT/q_smoke.log
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/q_pytest_gpu.log 2>&1 || { echo "pytest rc $?"; tail -40 $OUT/q_pytest_gpu.log; exit 1; }
tail -2 $OUT/q_pytest_gpu.log
echo "== bench (driver command)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/q_bench.log 2>&1 || { echo "bench rc $?"; tail -20 $OUT/q_bench.log; exit 1; }
grep '^{' $OUT/q_bench.log
