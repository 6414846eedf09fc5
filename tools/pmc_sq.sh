#!/usr/bin/env bash
# SQ issue/wait counters of the encode kernel under a few build switches
# (one rocprofv3 --pmc pass per setting; MI355X_MICROARCH.md §rocprofv3 PMC
# slots: 8 SQ + 1 GRBM per pass).  Usage: tools/pmc_sq.sh "ENV=.. ENV=.." ...
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_sq"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
i=0
for SETTING in "$@"; do
  i=$((i + 1))
  echo "== $i: $SETTING"
  # shellcheck disable=SC2086
  ( export $SETTING; timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$REPO/bench.py" --cpu-seconds 0 --e2e-stripes 0 --steps 20 --warmup 5 --verify 0 > "$OUT/p$i.log" 2>&1 )
  echo "$SETTING" > "$OUT/p$i/setting.txt"
  tail -1 "$OUT/p$i.log" | cut -c1-160
done
python3 "$REPO/tools/pmc_sq_summary.py" "$OUT"
