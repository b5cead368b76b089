#!/bin/bash
# round 4: k_scalar_inv fold by batch size (inv_small) -- parity suites that
# run host slices and small / large batches, then the c2_hostpath A/B
set -o pipefail
cd /root/repo
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_group_keys.py \
  tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 tools/hostpath_ab4.py 6 "pre:prestage=1" "nopre:prestage=0" > $O/ab.jsonl 2> $O/ab.err \
  || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4w/ab.jsonl')]
for n in dict.fromkeys(r['name'] for r in rows):
    rs=[r for r in rows if r['name']==n]
    print(n, 'pinned med', S.median(r['pinned'] for r in rs), [r['pinned'] for r in rs], 'pageable med', S.median(r['pageable'] for r in rs), [r['pageable'] for r in rs], 'bad', sum(r['pinned_bad']+r['pageable_bad'] for r in rs))
PY
