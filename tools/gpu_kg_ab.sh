#!/bin/bash
# Round 6: the grouped route's many-group ladders (option "kg") -- the ladder
# variant tests, then the headline alternated over GV_KG=0 (k4) / 6 / 7 / 9.
# usage: tools/gpu_kg_ab.sh OUT [reps] [variants...]
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/kg_ab}; REPS=${2:-2}; shift 2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ladder_variants.py \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
V=("$@"); [ ${#V[@]} -eq 0 ] && V=("k4:GV_KG=0" "kg6:GV_KG=6" "kg7:GV_KG=7" "kg9:GV_KG=9")
bash tools/gpu_ab_env.sh $OUT $REPS "${V[@]}"
