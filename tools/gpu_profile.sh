#!/usr/bin/env bash
# rocprofv3 passes over the bench: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md §HBM / §rocprofv3).
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof"
CFG="${1:-10+4@1MiB}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "== kernel trace"
# 1000 timed steps, so the 50 warm-up launches (and the post-idle clock
# ramp in them) move the --stats average by well under 1 %
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --config "$CFG" --cpu-seconds 0 --e2e-stripes 0 --steps 1000 > "$OUT/kt_bench.log" 2>&1
tail -1 "$OUT/kt_bench.log"
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 400 rocprofv3 --pmc "$C" -d "$OUT/pmc_$C" -o pmc --output-format csv -- \
      python3 "$REPO/bench.py" --config "$CFG" --cpu-seconds 0 --e2e-stripes 0 --steps 5 --warmup 1 --verify 0 > "$OUT/pmc_$C.log" 2>&1
  tail -1 "$OUT/pmc_$C.log" | cut -c1-200
done
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== calibration pmc $C (known bytes, 16- and 8-byte lanes)"
  timeout -k 10 200 rocprofv3 --pmc "$C" -d "$OUT/calib_$C" -o pmc --output-format csv -- \
      python3 "$REPO/tools/fetch_calib.py" > "$OUT/calib_$C.log" 2>&1
  tail -1 "$OUT/calib_$C.log" | cut -c1-200
done
find "$OUT" -name "*.csv" | head -20
