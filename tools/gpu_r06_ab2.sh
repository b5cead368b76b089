#!/bin/bash
# Round 6: the GPU tests the round's changes touch (async queue on gv_async.h,
# the split key chain, the kg layouts, the ladder's G frame), then the headline
# A/B: k4 vs kg4 (k4 tables, G after the ladder on the real curve) vs the
# unsplit key chain.
set -o pipefail
cd /root/repo
OUT=gpurun_out/r06_ab2; mkdir -p $OUT
L=cosmos-sdk-rootchain_amd/lib
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_async.py \
  tests/test_ladder_variants.py tests/test_key_cache.py tests/test_group_keys.py tests/test_hbm_budget.py \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/gpu_ab_env.sh $OUT 2 k4:GV_KG=0 kg4:GV_KG=4 "nosplit:GV_LIB=$L/libgpuverify_nosplit.so GV_KG=0"
