#!/bin/bash
# round 4: host-path A/B of slice_plain_first, more reps
set -o pipefail
cd /root/repo
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 700 python3 tools/hostpath_ab4.py 4 "off:slice_plain_first=0" "p128k:slice_plain_first=131072" \
  "p192k:slice_plain_first=196608" "p256k:slice_plain_first=262144" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4i/ab.jsonl')]
for n in dict.fromkeys(r['name'] for r in rows):
    rs=[r for r in rows if r['name']==n]
    print(n, 'pinned med', S.median(r['pinned'] for r in rs), [r['pinned'] for r in rs], 'pageable med', S.median(r['pageable'] for r in rs), 'bad', sum(r['pinned_bad']+r['pageable_bad'] for r in rs))
PY
