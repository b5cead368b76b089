#!/bin/bash
# round 4: key tables + key parse square root on the fused products -- parity,
# then C2 (bench, alternated) and c2_hostpath against the classic-product build
set -o pipefail
cd /root/repo
O=gpurun_out/r4ad; mkdir -p $O
L=/root/repo/cosmos-sdk-rootchain_amd/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_ladder_variants.py tests/test_key_cache.py tests/test_kat_gpu.py tests/test_group_keys.py > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh $O 3 "fused:GV_DUMMY=1" "classic:GV_LIB=$L/libgpuverify_old.so" || exit 1
for rep in 1 2; do
  for v in fused classic; do
    lib=$L/libgpuverify.so; [ $v = classic ] && lib=$L/libgpuverify_old.so
    GV_LIB=$lib timeout -k 10 300 python3 tools/hostpath_ab4.py 2 "$v:" > $O/hp_${v}_$rep.jsonl 2>> $O/hp.err || { tail -20 $O/hp.err; exit 1; }
    python3 -c "
import json, statistics as S
rs=[json.loads(l) for l in open('$O/hp_${v}_$rep.jsonl')]
print('$v', 'hostpath pinned', [r['pinned'] for r in rs], 'pageable', [r['pageable'] for r in rs])"
  done
done
