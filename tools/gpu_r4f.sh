#!/bin/bash
# round 4: kernel trace + stats of the default bench (k4 ladder, full-scalar G)
set -o pipefail
O=/root/repo/gpurun_out/r4f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- \
  python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency > $O/trace.json 2>$O/trace.err \
  || { tail -20 $O/trace.err; exit 1; }
python3 /root/repo/tools/prof_timed.py $O/trace/t_kernel_trace.csv 10 $O/timed.csv > $O/timed.txt
cat $O/timed.txt
