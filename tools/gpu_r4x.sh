#!/bin/bash
# round 4: lambda-frame switch in the k4 ladder (GV_LAMFRAME) -- parity, then
# the C2 A/B against the per-entry beta product build
set -o pipefail
cd /root/repo
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_group_keys.py tests/test_ladder_variants.py tests/test_key_cache.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=/root/repo/cosmos-sdk-rootchain_amd/lib
bash tools/gpu_ab_env.sh $O 3 "lamframe:GV_DUMMY=1" "perentry:GV_LIB=$L/libgpuverify_lam0.so" || exit 1
