# The k6-family ladders' G tables at 26-bit windows (make ab NAME=g26
# DEFS=-DGV_K6_GW=26: 10 tables of 2^25 entries, 21.5 GB, 10 G additions)
# against the default 24-bit build: the tests that run those ladders, then
# c2_key_cache (kw / kw2 / kn) and gv_open's time, alternated.
set -o pipefail
cd /root/repo
O=${1:-gpurun_out/g26}; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
GV_LIB=$L/libgpuverify_g26.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ladder_variants.py tests/test_key_cache.py tests/test_hbm_budget.py tests/test_gpu_parity.py ${EXTRA_TESTS:-} > $O/tests_g26.log 2>&1 || { tail -30 $O/tests_g26.log; exit 1; }
tail -2 $O/tests_g26.log
for i in 1 2; do
  for v in g26 g24; do
    lib=$L/libgpuverify_$v.so; [ $v = g24 ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 240 python -u tools/kw_ab.py 1 > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    cut -c1-200 $O/${v}_$i.jsonl | sed "s/^/$v $i: /"
  done
done
