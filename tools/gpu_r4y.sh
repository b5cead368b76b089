#!/bin/bash
# round 4: k_ecmult_k4 kernel durations, lambda-frame vs per-entry beta (rocprofv3 stats, alternated)
set -o pipefail
O=/root/repo/gpurun_out/r4y; mkdir -p $O
L=/root/repo/cosmos-sdk-rootchain_amd/lib
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in lamframe perentry; do
    lib=$L/libgpuverify.so; [ $v = perentry ] && lib=$L/libgpuverify_lam0.so
    GV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${v}_$rep -o run -- \
      python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency \
      > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -20 $O/b_${v}_$rep.err; exit 1; }
    python3 - $O/p_${v}_$rep $v $O/b_${v}_$rep.json <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'ecmult_k4' in r['Name']:
        print(sys.argv[2], 'k4 avg ms', round(float(r['AverageNs']) / 1e6, 4), 'calls', r['Calls'], 'value', round(json.load(open(sys.argv[3]))['value'] / 1e6, 2))
PY
  done
done
