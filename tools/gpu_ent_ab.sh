set -o pipefail
O=gpurun_out/ent; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
GV_LIB=$L/libgpuverify_ent32.so timeout -k 10 400 python -u -m pytest tests/test_ladder_variants.py -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -k "cached or wide" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in base ent32; do
    lib=$L/libgpuverify_$v.so; [ $v = base ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 200 python -u tools/kw_ab.py 1 > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    head -2 $O/${v}_$i.jsonl | cut -c1-150 | sed "s/^/$v $i: /"
  done
done
