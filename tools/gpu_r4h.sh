#!/bin/bash
# round 4: the plain-first-chunk option (parity + host-path A/B)
set -o pipefail
cd /root/repo
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_group_keys.py \
  tests/test_ladder_variants.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python3 tools/hostpath_ab4.py 2 "off:slice_plain_first=0" "p64k:slice_plain_first=65536" \
  "p128k:slice_plain_first=131072" "p192k:slice_plain_first=196608" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
