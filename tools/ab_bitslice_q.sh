#!/usr/bin/env bash
# A/B: bit-sliced kernel with 8-byte pieces (default) vs 16-byte pieces
# (var=202) vs the perm-table kernels (bitslice=0); bitslice=2 puts the
# 4-parity shapes on the bit-sliced kernel too.
set -e
for km in "10 8" "10 6" "8 5"; do
  set -- $km
  echo "== $1+$2 encode"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "var=202" "bitslice=0"
done
for km in "10 4" "12 4"; do
  set -- $km
  echo "== $1+$2 encode"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "bitslice=2" "bitslice=2,var=202"
done
