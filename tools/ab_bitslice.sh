#!/usr/bin/env bash
# A/B: bit-sliced Encode (default for the generated shapes) vs the perm-table
# kernels (bitslice=0), split layout, 1 MiB vectors (tools/ab.py).
set -e
for km in "10 8" "10 6" "10 5" "12 8" "8 5" "8 8"; do
  set -- $km
  echo "== $1+$2 encode"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "bitslice=0"
done
