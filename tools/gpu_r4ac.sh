#!/bin/bash
# round 4: lambda frame with one switch per position (GV_LAMFRAME=2) vs two (1):
# parity, then C2 bench alternated and the rocprofv3-timed ladder
set -o pipefail
cd /root/repo
O=gpurun_out/r4ac; mkdir -p $O
L=/root/repo/cosmos-sdk-rootchain_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_ladder_variants.py tests/test_key_cache.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh $O 3 "lf2:GV_DUMMY=1" "lf1:GV_LIB=$L/libgpuverify_lf1.so" || exit 1
cd /tmp && export TMPDIR=/tmp
for v in lf2 lf1; do
  lib=$L/libgpuverify.so; [ $v = lf1 ] && lib=$L/libgpuverify_lf1.so
  GV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- \
    python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency \
    > $O/bp_$v.json 2> $O/bp_$v.err || { tail -20 $O/bp_$v.err; exit 1; }
  python3 /root/repo/tools/prof_timed.py $O/p_$v/run_kernel_trace.csv 10 $O/kt_$v.csv > /dev/null
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kt_$v.csv')):
    if 'ecmult_k4' in r['Name']: print('$v k4 timed ms', round(float(r['TimedAverageNs'])/1e6, 4))"
done
