#!/bin/bash
# round 4: host-path chunk ramp re-swept on the full-scalar-G ladder
set -o pipefail
cd /root/repo
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 900 python3 tools/hostpath_ab4.py 3 "c262g4:pipe_chunk=262144,pipe_growth=4" \
  "c262g1:pipe_chunk=262144,pipe_growth=1" "c196g2:pipe_chunk=196608,pipe_growth=2" \
  "c131g2:pipe_chunk=131072,pipe_growth=2" "c334g1:pipe_chunk=334080,pipe_growth=1" > $O/ab.jsonl 2> $O/ab.err \
  || { tail -20 $O/ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S
rows=[json.loads(l) for l in open('gpurun_out/r4j/ab.jsonl')]
for n in dict.fromkeys(r['name'] for r in rows):
    rs=[r for r in rows if r['name']==n]
    print(n, 'pinned med', S.median(r['pinned'] for r in rs), [r['pinned'] for r in rs], 'pageable med', S.median(r['pageable'] for r in rs), [r['pageable'] for r in rs], 'bad', sum(r['pinned_bad']+r['pageable_bad'] for r in rs))
PY
