#!/usr/bin/env bash
# The committed profiles of the headline kernel, one GPU call per round:
#  1. the driver's own command under rocprofv3 --kernel-trace --stats, and
#     tools/trace_window.py cutting its timed window out (the headline kernel
#     alone, no end-to-end or self-check launches)
#  2. tools/gpu_profile.sh: kernel trace of a 1000-step bench without the
#     end-to-end leg, FETCH_SIZE / WRITE_SIZE passes and their calibration
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof_driver"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT" -o drv --output-format csv -- \
    python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
grep '^{' "$OUT/bench.log" | cut -c1-200
TRACE=$(find "$OUT" -name "drv_kernel_trace.csv" | head -1)
python3 "$REPO/tools/trace_window.py" "$TRACE" "$OUT/bench.log" "$OUT/trace_window.json" "$OUT/timed_window_stats.csv" | head -30
bash "$REPO/tools/gpu_profile.sh"
