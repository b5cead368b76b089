# The resident arena at wider windows (make ab NAME=k10 / k11 DEFS=-DGV_KW_QW=10 / 11)
# against the default 9-bit build: one variant's keyed / ladder tests (TESTLIB),
# then c2_key_cache alternated over VARIANTS (tools/kw_ab.py).
set -o pipefail
cd /root/repo
O=${1:-gpurun_out/kq10}; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
GV_LIB=$L/libgpuverify_${TESTLIB:-k10}.so timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ladder_variants.py tests/test_key_cache.py > $O/tests_${TESTLIB:-k10}.log 2>&1 || { tail -30 $O/tests_${TESTLIB:-k10}.log; exit 1; }
tail -2 $O/tests_${TESTLIB:-k10}.log
for i in 1 2; do
  for v in ${VARIANTS:-k10 k9}; do
    lib=$L/libgpuverify_$v.so; [ $v = k9 ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 240 python -u tools/kw_ab.py 1 > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    cut -c1-230 $O/${v}_$i.jsonl | sed "s/^/$v $i: /"
  done
done
