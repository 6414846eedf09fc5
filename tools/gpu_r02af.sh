#!/usr/bin/env bash
# Round-2 GPU pass af: SQ counters of 10+8 Reconst of 8 lost, run-time
# bit-sliced kernel vs perm-table kernel (one rocprofv3 --pmc pass each).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_sq_jit"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
i=0
for SETTING in "op=rec8,jit=2" "op=rec8,jit=0" "op=enc,jit=2" ; do
  i=$((i + 1))
  K=10; [ "$SETTING" = "op=enc,jit=2" ] && K=16
  echo "== $i: $SETTING (k=$K)"
  AB_K=$K AB_M=8 AB_ROUNDS=2 AB_ITERS=5 timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$REPO/tools/ab.py" "$SETTING" > "$OUT/p$i.log" 2>&1 || { echo "rc $?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "$SETTING k=$K" > "$OUT/p$i/setting.txt"
  grep median "$OUT/p$i.log" | cut -c1-120
done
python3 "$REPO/tools/pmc_sq_summary.py" "$OUT"
