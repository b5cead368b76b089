#!/bin/bash
# Round 6 A/B 3: kn ladders with zq parked in LDS (GV_KN_ZQ_LDS: 4 waves per
# SIMD) on the grouped route's kg layouts vs k4, and on the resident arena
# (kw / kw2 / kn) with and without the entry prefetch (GV_KN_PREFETCH).
set -o pipefail
cd /root/repo
OUT=gpurun_out/r06_ab3; mkdir -p $OUT
L=cosmos-sdk-rootchain_amd/lib
bash tools/gpu_ab_env.sh $OUT 2 k4:GV_KG=0 "kg4z:GV_LIB=$L/libgpuverify_zqlds.so GV_KG=4" \
  "kg7z:GV_LIB=$L/libgpuverify_zqlds.so GV_KG=7" "kg9z:GV_LIB=$L/libgpuverify_zqlds.so GV_KG=9" \
  "nosplit:GV_LIB=$L/libgpuverify_nosplit.so GV_KG=0" || exit 1
for i in 1 2; do
  for v in base knpf zqlds zqldspf; do
    lib=$L/libgpuverify_$v.so; [ $v = base ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 300 python -u tools/kw_ab.py 1 > $OUT/kw_${v}_$i.jsonl 2> $OUT/kw_${v}_$i.err || { tail -20 $OUT/kw_${v}_$i.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/kw_${v}_$i.jsonl'):
    d = json.loads(l); print('$v', $i, d['keys_wide'], d['route'], round(d['value'] / 1e6, 1), 'ladder', d['ladder_ms'], 'mm', d['mismatches'])"
  done
done
