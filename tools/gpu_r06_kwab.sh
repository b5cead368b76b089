#!/bin/bash
# Round 6: the resident arena's ladders (kw / kw2 / kn) with the one-slot-ahead
# entry prefetch (GV_KN_PREFETCH=1 build) against the default, alternated in
# processes of their own; then the kw tests on the prefetch build.
set -o pipefail
cd /root/repo
OUT=gpurun_out/r06_kwab; mkdir -p $OUT
L=cosmos-sdk-rootchain_amd/lib
for i in 1 2; do
  for v in base knpf; do
    lib=$L/libgpuverify.so; [ $v = knpf ] && lib=$L/libgpuverify_knpf.so
    GV_LIB=$lib timeout -k 10 300 python -u tools/kw_ab.py 1 > $OUT/${v}_$i.jsonl 2> $OUT/${v}_$i.err || { tail -20 $OUT/${v}_$i.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/${v}_$i.jsonl'):
    d = json.loads(l); print('$v', $i, d['keys_wide'], d['route'], round(d['value'] / 1e6, 1), 'ladder', d['ladder_ms'], 'mm', d['mismatches'])"
  done
done
GV_LIB=$L/libgpuverify_knpf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_ladder_variants.py -k "cached or wide" > $OUT/tests_knpf.log 2>&1 || { tail -30 $OUT/tests_knpf.log; exit 1; }
tail -2 $OUT/tests_knpf.log
