#!/usr/bin/env bash
# HBM traffic and SQ occupancy of the shipped wide networks (verdict round 3,
# item 3: traffic <= 1.10x algorithmic): for each tools/pmc_traffic.py spec
# given (e.g. enc:64+64), one rocprofv3 --pmc pass for FETCH_SIZE and one for
# WRITE_SIZE (MI355X_MICROARCH.md §HBM: separate passes), then one calibration
# pass per counter over known bytes (tools/fetch_calib.py), then the SQ passes
# of tools/pmc_icache.sh.  Summaries: gpurun_out/pmc_wide/traffic_<tag>.json
# and gpurun_out/pmc_icache/summary.json.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_wide"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/calib_$C" -o pmc --output-format csv -- \
      python3 "$REPO/tools/fetch_calib.py" > "$OUT/calib_$C.log" 2>&1 || { echo "calib $C failed"; exit 1; }
done
for SPEC in "$@"; do
  tag="${SPEC//[:+@=,]/_}"
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== $SPEC $C"
    timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/${tag}_$C" -o pmc --output-format csv -- \
        python3 "$REPO/tools/pmc_traffic.py" run "$SPEC" > "$OUT/${tag}_$C.log" 2>&1 || { echo "pass failed"; tail -5 "$OUT/${tag}_$C.log"; exit 1; }
  done
  alg=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['algorithmic_bytes_per_launch'])" "$OUT/${tag}_FETCH_SIZE.log")
  python3 "$REPO/tools/pmc_traffic.py" summarize "$SPEC" "$OUT/${tag}_FETCH_SIZE" "$OUT/${tag}_WRITE_SIZE" \
      "$OUT/calib_FETCH_SIZE" "$OUT/calib_WRITE_SIZE" "$alg" | tee "$OUT/traffic_$tag.json"
done
[ "${PMC_WIDE_SQ:-1}" = 0 ] || bash "$REPO/tools/pmc_icache.sh" "$@"
