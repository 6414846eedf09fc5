#!/usr/bin/env bash
# Round-2 GPU pass ai: default kernel after moving the XCD remap into an
# experimental variant (var=160): A/B and the driver's bench command.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -u tools/ab.py "var=-1" "var=160" > "$OUT/ab_ai.log" 2>&1 || { tail -20 "$OUT/ab_ai.log"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_ai.log"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/ai_bench.log 2>&1 || { echo "bench rc $?"; tail -20 $OUT/ai_bench.log; exit 1; }
grep '^{' $OUT/ai_bench.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "encode or bench" > "$OUT/ai_pytest.log" 2>&1 || { tail -30 "$OUT/ai_pytest.log"; exit 1; }
tail -1 "$OUT/ai_pytest.log"
