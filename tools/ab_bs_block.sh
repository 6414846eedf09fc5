#!/usr/bin/env bash
# A/B of the bit-sliced Encode's workgroup size (rs_tune bs_block: 0 = the
# per-layout rule, 64 / 128 / 256 forced) on the split and interleaved layouts.
set -e
for km in "10 8" "10 6" "12 8" "8 5" "10 5" "8 8"; do
  set -- $km
  echo "== $1+$2 encode, split"
  AB_K=$1 AB_M=$2 AB_ROUNDS=6 timeout -k 10 200 python -u tools/ab.py "" "bs_block=64" "bs_block=128" "bs_block=256"
  echo "== $1+$2 encode, interleaved"
  AB_K=$1 AB_M=$2 AB_ROUNDS=6 timeout -k 10 200 python -u tools/ab.py "layout=inter" "bs_block=64,layout=inter" \
      "bs_block=128,layout=inter" "bs_block=256,layout=inter"
done
