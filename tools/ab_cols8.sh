#!/usr/bin/env bash
# A/B of the generic kernels' column batch: default (8-column batches for 5-8
# columns, 4 above) vs var=200 (8-column batches above 8 columns too), and the
# old 4-column batches via max_grid (looped kernel) for reference (tools/ab.py).
set -e
for km in "16 4" "14 4" "9 3" "12 4" "20 4" "16 8"; do
  set -- $km
  echo "== $1+$2 encode / reconst"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "var=200" "op=rec1" "op=rec1,var=200"
done
