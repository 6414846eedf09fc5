#!/usr/bin/env bash
# A/B of the 5-8-output-row kernels: one-chunk (default) vs the looped kernel
# (max_grid forces it) vs 8-column batches (var=200), Encode and Replace of 3
# rows (tools/ab.py).
set -e
for km in "10 8" "12 8" "8 5" "16 8" "20 6"; do
  set -- $km
  echo "== $1+$2 encode / replace3"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "max_grid=1073741824" "var=200" "op=rep3" "op=rep3,var=200" "op=rep3,max_grid=1073741824"
done
