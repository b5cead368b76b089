#!/bin/bash
# round 4: ed25519 products with the high-column mad carry (parity + A/B)
set -o pipefail
cd /root/repo
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ed_gpu.py \
  tests/test_ed_keyed_gpu.py tests/test_ibc_commits.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in hc classic; do
    env_lib=""
    [ $v = classic ] && env_lib="GV_LIB=/root/repo/cosmos-sdk-rootchain_amd/lib/libgpuverify_e29c.so"
    env $env_lib timeout -k 10 240 python3 tools/ed_probe.py 1000000 16 > $O/ed_${v}_$rep.json 2>> $O/ed.err || { tail -20 $O/ed.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ed_${v}_$rep.json')); print('$v', $rep, round(d['value']/1e6,2), d.get('mismatches'), {k: (v if not isinstance(v, dict) else '') for k, v in d.items() if k in ('throughput_value','keyed_value','value_throughput')})"
  done
done
