#!/bin/bash
# A/B of the wide arena's windows per group: libgpuverify_wpg1 (make ab
# NAME=wpg1 DEFS=-DGV_KW_WPG=1: one window per group, no doublings) against the
# default (two per group, 9 doublings); parity first, then c2_key_cache
# alternated, each in a process of its own.
set -o pipefail
O=gpurun_out/wpg; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
GV_LIB=$L/libgpuverify_wpg1.so timeout -k 10 400 python -u -m pytest tests/test_ladder_variants.py tests/test_key_cache.py -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -k "cached or wide or keyed" > $O/tests_wpg1.log 2>&1; rc=$?; tail -3 $O/tests_wpg1.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in wpg2 wpg1; do
    lib=$L/libgpuverify_$v.so; [ $v = wpg2 ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 200 python -u tools/kw_ab.py 1 > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    head -1 $O/${v}_$i.jsonl | cut -c1-190 | sed "s/^/$v $i: /"
  done
done
