#!/bin/bash
# round 4: secp classic products with the high-column mad carry (parity + A/B)
set -o pipefail
cd /root/repo
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_group_keys.py tests/test_kat_gpu.py tests/test_key_cache.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=/root/repo/cosmos-sdk-rootchain_amd/lib
bash tools/gpu_ab_env.sh $O 2 "hc:GV_DUMMY=1" "classic:GV_LIB=$L/libgpuverify_f29c.so" || exit 1
for v in hc classic; do
  env_lib=""; [ $v = classic ] && env_lib="GV_LIB=$L/libgpuverify_f29c.so"
  env $env_lib timeout -k 10 200 python3 - > $O/uk_$v.json 2>>$O/uk.err <<'PY' || exit 1
import json, sys
sys.path[:0] = ['/root/repo', '/root/repo/cosmos-sdk-rootchain_amd', '/root/repo/tools']
import bench, bench_extras as X, gpuverify as gvm
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
ver = gvm.Verifier([0])
r = X.c2_per_item_parse(ver, pub, sig, dig, exp)
print(json.dumps({"per_item": r["value"], "stages": r["stages"], "mismatches": r["mismatches"]}))
PY
  echo $v; cat $O/uk_$v.json
done
