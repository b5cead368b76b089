#!/bin/bash
# round 4 end: full GPU suite, the default bench (with extras), then a
# kernel-trace + stats profile of the headline bench command.  Every GPU step
# has its own limit; the chain stops at the first failure.
set -o pipefail
cd /root/repo
O=gpurun_out/r4end; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; b=json.load(open('$O/bench.json')); print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['kernel_ms'], b.get('checktx_p50_ms_64'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$O/prof -o run -- \
  python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency \
  > /root/repo/$O/bench_prof.json 2> /root/repo/$O/bench_prof.err || { tail -20 /root/repo/$O/bench_prof.err; exit 1; }
python3 /root/repo/tools/prof_timed.py /root/repo/$O/prof/run_kernel_trace.csv 10 /root/repo/$O/kernel_timed.csv > /root/repo/$O/timed.txt; head -12 /root/repo/$O/timed.txt
