#!/bin/bash
# round 4: full-scalar G windows on k4 -- parity of every ladder schedule, then A/B gfull 1/0
set -o pipefail
cd /root/repo
OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ladder_variants.py \
  tests/test_group_keys.py tests/test_sort_keys.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/gpu_ab_env.sh $OUT 2 "gf:GV_GFULL=1" "glv:GV_GFULL=0"
