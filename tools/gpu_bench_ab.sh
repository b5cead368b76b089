#!/bin/bash
# Headline bench (no extras) A/B: the default library against
# cosmos-sdk-rootchain_amd/lib/libgpuverify_$1.so, alternated, each run in a
# process of its own.  usage: gpu_bench_ab.sh NAME [reps]
set -o pipefail
V=$1; R=${2:-3}
O=gpurun_out/bench_ab_$V; mkdir -p $O
L=cosmos-sdk-rootchain_amd/lib
for i in $(seq 1 $R); do
  for v in base $V; do
    lib=$L/libgpuverify_$v.so; [ $v = base ] && lib=$L/libgpuverify.so
    GV_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-extras > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1])
print('$v $i', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms/step ladder', d['roofline']['kernel_ms'], 'front', d['pipeline']['scalar_inv_ms'])"
  done
done
