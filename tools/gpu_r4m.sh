#!/bin/bash
# round 4: pageable chunks staged in pieces (parity + host-path A/B)
set -o pipefail
cd /root/repo
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_group_keys.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 700 python3 tools/hostpath_ab4.py 3 "p4:stage_pieces=4" "p1:stage_pieces=1" "p8:stage_pieces=8" "p2:stage_pieces=2" \
  > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4m/ab.jsonl')]
for n in dict.fromkeys(r['name'] for r in rows):
    rs=[r for r in rows if r['name']==n]
    print(n, 'pinned med', S.median(r['pinned'] for r in rs), 'pageable med', S.median(r['pageable'] for r in rs), [r['pageable'] for r in rs], 'bad', sum(r['pinned_bad']+r['pageable_bad'] for r in rs))
PY
