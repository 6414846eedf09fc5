#!/usr/bin/env bash
# Instruction supply of the run-time compiled networks (verdict round 3,
# item 3): SQ issue / wait and instruction-fetch counters and the SQC
# instruction-cache counters of the rs_bs_asm kernel, one rocprofv3 --pmc pass
# per counter group (MI355X_MICROARCH.md §rocprofv3 PMC slots), for each
# shape given (tools/pmc_traffic.py specs, e.g. enc:64+64).  Summary:
# gpurun_out/pmc_icache/summary.json (tools/pmc_sq_summary.py).  PMC_GROUPS
# picks the counter groups (default "SQ SQC"; "LDS" = the wait / LDS split;
# "VALU" = SIMD VALU cycles against the waves').
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/${PMC_OUT:-pmc_icache}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_IFETCH SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE"
SQC="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
# LDS: where parked / stalled cycles come from (s_waitcnt + barrier vs LDS issue stalls and bank conflicts)
LDS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
# VALU: SIMD-side VALU cycles against the waves' (is the SIMD or the wave the limit?)
VALU="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for SPEC in "$@"; do
  for GROUP in ${PMC_GROUPS:-SQ SQC}; do
    i=$((i + 1))
    CTRS="${!GROUP}"
    echo "== p$i: $SPEC $GROUP"
    # shellcheck disable=SC2086
    timeout -s KILL 90 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
        python3 "$REPO/tools/pmc_traffic.py" run "$SPEC" > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "$SPEC $GROUP" > "$OUT/p$i/setting.txt" 2>/dev/null || true
    tail -2 "$OUT/p$i.log" | cut -c1-200
    if [ $rc -ne 0 ]; then echo "pass p$i failed rc=$rc"; exit $rc; fi
  done
done
python3 "$REPO/tools/pmc_sq_summary.py" "$OUT"
