#!/bin/bash
# round 4: host-mirror GPU tests after the miss split, then C1 / C4 (default settings, 6 reps)
set -o pipefail
cd /root/repo
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_paths.py \
  tests/test_ante_mirror.py tests/test_gas_order.py tests/test_amino_decode.py -m gpu > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 700 python3 -u tools/mirror_ab.py 6 30000 12 cur:GVH_DEFER_RELEASE=1 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4z/ab.jsonl')]
for n in dict.fromkeys(r['name'] for r in rows):
    rs=[r for r in rows if r['name']==n]
    print(n, {k: (S.median(r[k] for r in rs), [r[k] for r in rs]) for k in rs[0] if k not in ('rep','name')})
PY
