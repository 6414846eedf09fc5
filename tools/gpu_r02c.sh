#!/usr/bin/env bash
# Round-2 GPU pass c: new parity tests (compat mode, lane-group kernels, full
# size every stripe), lane-group A/B, driver bench + rocprof.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
echo "== new parity tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "row_group or parity_rows_bitsliced or compat_mode or full_size" > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -2 "$OUT/pytest_new.log"
echo "== A/B lane groups"
AB_K=10 AB_M=8 AB_ROUNDS=8 timeout -k 10 300 python -u tools/ab.py "op=rec8,rg4=0" "op=rec8,rg4=1" "op=rec8,rg4=2" \
    "op=rec5,rg4=0" "op=rec5,rg4=1" "op=rec5,rg4=2" "bitslice=0,rg4=0" "bitslice=0,rg4=1" "bitslice=1" \
    2>&1 | grep -v amdgpu.ids | tee "$OUT/ab_rgw_10_8.log"
AB_K=16 AB_M=8 AB_ROUNDS=8 timeout -k 10 300 python -u tools/ab.py "rg4=0" "rg4=1" "rg4=2" "op=rec8,rg4=0" "op=rec8,rg4=1" \
    2>&1 | grep -v amdgpu.ids | tee "$OUT/ab_rgw_16_8.log"
echo "== driver bench command"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || { tail -20 "$OUT/bench_driver.log"; exit 1; }
grep '^{' "$OUT/bench_driver.log" | cut -c1-300
echo "== driver bench command under rocprofv3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_prof.log" 2>&1 || { tail -20 "$OUT/bench_driver_prof.log"; exit 1; }
grep '^{' "$OUT/bench_driver_prof.log" | cut -c1-300
