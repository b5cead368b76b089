#!/bin/bash
# round 4: kernel trace + stats of the headline bench command, the PMC passes
# (tools/pmc_round.sh) and the host-path A/B of slice_plain_first.
set -o pipefail
cd /root/repo
O=gpurun_out/r4prof; mkdir -p $O
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /root/repo/$O/prof -o run -- python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline \
    --no-latency > /root/repo/$O/bench_prof.json 2> /root/repo/$O/bench_prof.err ) || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/prof_timed.py $O/prof/run_kernel_trace.csv 10 $O/kernel_timed.csv | head -8
bash tools/pmc_round.sh $O/pmc 1000000 || exit 1
python3 tools/pmc_summary.py $O/pmc 1000000 $O/pmc_summary.json > $O/pmc_summary.txt 2>&1 || true
tail -5 $O/pmc_summary.txt
timeout -k 10 400 python3 tools/hostpath_ab4.py 2 "off:slice_plain_first=0" "p64k:slice_plain_first=65536" \
  "p128k:slice_plain_first=131072" > $O/hp_ab.jsonl 2> $O/hp_ab.err || { tail -20 $O/hp_ab.err; exit 1; }
cat $O/hp_ab.jsonl
