#!/bin/bash
# C1 one-block-at-a-time A/B: this tree's libraries vs a round-4 build staged
# under ab_r04/ (not tracked), alternated, each run in a process of its own.
set -o pipefail
O=gpurun_out/c1ab; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python3 tools/c1_probe.py 10000 8 16 > $O/head_$i.txt 2>&1 || { tail $O/head_$i.txt; exit 1; }
  grep -E "steady|block 8" $O/head_$i.txt | sed "s/^/head $i: /"
  ( cd ab_r04 && timeout -k 10 120 python3 tools/c1_probe.py 10000 8 16 ) > $O/r04_$i.txt 2>&1 || { tail $O/r04_$i.txt; exit 1; }
  grep -E "steady|block 8" $O/r04_$i.txt | sed "s/^/r04 $i: /"
done
