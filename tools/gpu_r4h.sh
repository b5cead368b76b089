#!/bin/bash
# round 4: host-path timelines, the plain-first-chunk option (parity + A/B)
set -o pipefail
cd /root/repo
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_group_keys.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 tools/hostpath_ab4.py 3 "off:slice_plain_first=0" "p64k:slice_plain_first=65536" \
  "p128k:slice_plain_first=131072" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
cd /tmp && export TMPDIR=/tmp
for m in pinned pageable; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /root/repo/$O/tr_$m -o t -- \
    python3 /root/repo/tools/hostpath_trace.py /root/repo/$O/calls_$m.json $m 3 > /root/repo/$O/run_$m.txt 2>&1 \
    || { tail -20 /root/repo/$O/run_$m.txt; exit 1; }
  python3 /root/repo/tools/hostpath_trace.py --analyze /root/repo/$O/tr_$m /root/repo/$O/calls_$m.json > /root/repo/$O/an_$m.txt 2>&1
  head -40 /root/repo/$O/an_$m.txt
done
