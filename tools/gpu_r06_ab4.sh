#!/bin/bash
# Round 6 A/B 4: the new defaults (grouped route on kg 4 -- k4 tables, G after
# the ladder on the real curve, zq in LDS, 4 waves per SIMD -- and the unsplit
# key chain) against k4 (GV_KG=0) and against the split chain; the GPU tests of
# the touched paths first.
set -o pipefail
cd /root/repo
OUT=gpurun_out/r06_ab4; mkdir -p $OUT
L=cosmos-sdk-rootchain_amd/lib
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ladder_variants.py \
  tests/test_hbm_budget.py tests/test_group_keys.py tests/test_sort_keys.py tests/test_key_cache.py \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_ab_env.sh $OUT 3 kg4:GV_KG=4 k4:GV_KG=0 "kg4split:GV_LIB=$L/libgpuverify_split.so GV_KG=4"
