#!/bin/bash
# round 4: gpu_hash (sign bytes hashed in the GPU batch) -- host-mirror GPU
# tests, then the C1 / C4 A/B
set -o pipefail
cd /root/repo
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_paths.py \
  tests/test_ante_mirror.py tests/test_gas_order.py tests/test_amino_decode.py -m gpu > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python3 -u tools/gpuhash_ab.py 4 30000 12 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4q/ab.jsonl')]
for gh in (True, False):
    rs=[r for r in rows if r['gpu_hash']==gh]
    print('gpu_hash', gh, {k: (S.median(r[k] for r in rs), [r[k] for r in rs]) for k in rs[0] if k not in ('rep','gpu_hash')})
PY
