#!/bin/bash
# A/B of the resident arena's wide-window width: libgpuverify_k7 / _k8 (make ab
# NAME=k7 DEFS=-DGV_KW_QW=7, ...) against the default build (QW 9), each in a
# process of its own, alternated.
set -o pipefail
O=gpurun_out/kq; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
for i in 1 2; do
  for v in k7 k8 k9; do
    lib=$L/libgpuverify_$v.so; [ $v = k9 ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 200 python -u tools/kw_ab.py 1 > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    head -1 $O/${v}_$i.jsonl | cut -c1-200 | sed "s/^/$v $i: /"
  done
done
