#!/bin/bash
# round 4: per-item Q table on the fused products -- parity, then the per-item
# C2 lines against the classic-product build, alternated
set -o pipefail
cd /root/repo
O=gpurun_out/r4ae; mkdir -p $O
L=/root/repo/cosmos-sdk-rootchain_amd/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_ladder_variants.py tests/test_kat_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in fused classic; do
    lib=$L/libgpuverify.so; [ $v = classic ] && lib=$L/libgpuverify_old.so
    GV_LIB=$lib timeout -k 10 300 python3 - $v >> $O/ab.jsonl 2>> $O/ab.err <<'PY' || exit 1
import json, sys
sys.path[:0] = ['/root/repo', '/root/repo/cosmos-sdk-rootchain_amd', '/root/repo/tools']
import bench, bench_extras as X, gpuverify as gvm
ver = gvm.Verifier([0])
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
pi = X.c2_per_item_parse(ver, pub, sig, dig, exp)
uk = X.c2_unique_keys(ver, bench.make_digest_workload, 1_000_000, 16)
print(json.dumps({"v": sys.argv[1], "per_item": round(pi["value"] / 1e6, 2), "unique": round(uk["value"] / 1e6, 2),
                  "mism": pi["mismatches"] + uk["mismatches"], "pi_prep_ms": pi["stages"]["prep_ms"], "uk_prep_ms": uk["stages"]["prep_ms"]}))
PY
    tail -1 $O/ab.jsonl
  done
done
