#!/bin/bash
# round 4: timelines of the c2 host path (pinned and pageable caller buffers)
set -o pipefail
O=/root/repo/gpurun_out/r4t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in pinned; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$m -o t -- \
    python3 /root/repo/tools/hostpath_trace.py $O/calls_$m.json $m 3 > $O/run_$m.txt 2>&1 || { tail -20 $O/run_$m.txt; exit 1; }
  cat $O/run_$m.txt | tail -2
  python3 /root/repo/tools/hostpath_trace.py --analyze $O/tr_$m $O/calls_$m.json > $O/an_$m.txt 2>&1
  head -70 $O/an_$m.txt
done
