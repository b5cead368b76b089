#!/bin/bash
# round 4: per-item route with G on the unsplit u1 (gfull_item) -- parity, then
# per-item C2 lines with the option on / off, alternated
set -o pipefail
cd /root/repo
O=gpurun_out/r4ab; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ladder_variants.py \
  tests/test_gpu_parity.py tests/test_group_keys.py tests/test_kat_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in 1 0; do
    GV_GFULL_ITEM=$v timeout -k 10 300 python3 - $v >> $O/ab.jsonl 2>> $O/ab.err <<'PY' || exit 1
import json, sys
sys.path[:0] = ['/root/repo', '/root/repo/cosmos-sdk-rootchain_amd', '/root/repo/tools']
import bench, bench_extras as X, gpuverify as gvm
ver = gvm.Verifier([0])
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
pi = X.c2_per_item_parse(ver, pub, sig, dig, exp)
uk = X.c2_unique_keys(ver, bench.make_digest_workload, 1_000_000, 16)
r = ver.route_stats()
print(json.dumps({"gfull_item": int(sys.argv[1]), "per_item": round(pi["value"] / 1e6, 2), "unique": round(uk["value"] / 1e6, 2),
                  "mism": pi["mismatches"] + uk["mismatches"], "item_f": r["item_f"], "pub33": r["pub33"],
                  "pi_ecmult_ms": pi["stages"]["ecmult_ms"], "uk_ecmult_ms": uk["stages"]["ecmult_ms"]}))
PY
    tail -1 $O/ab.jsonl
  done
done
