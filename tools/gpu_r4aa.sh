#!/bin/bash
# round 4: lambda entries in reverse group order (GV_LAMREV) vs forward --
# parity, timed ladder (rocprofv3 stats, alternated) and the ladder's FETCH_SIZE
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r4aa; mkdir -p $O
L=/root/repo/cosmos-sdk-rootchain_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_ladder_variants.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in rev fwd; do
    lib=$L/libgpuverify.so; [ $v = fwd ] && lib=$L/libgpuverify_fwd.so
    GV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${v}_$rep -o run -- \
      python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency \
      > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -20 $O/b_${v}_$rep.err; exit 1; }
    python3 /root/repo/tools/prof_timed.py $O/p_${v}_$rep/run_kernel_trace.csv 10 $O/kt_${v}_$rep.csv > /dev/null
    python3 - $O/kt_${v}_$rep.csv $v $O/b_${v}_$rep.json <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'ecmult_k4' in r['Name']:
        print(sys.argv[2], 'k4 timed ms', round(float(r['TimedAverageNs']) / 1e6, 4), 'value', round(json.load(open(sys.argv[3]))['value'] / 1e6, 2))
PY
  done
done
for v in rev fwd; do
  lib=$L/libgpuverify.so; [ $v = fwd ] && lib=$L/libgpuverify_fwd.so
  GV_LIB=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $O/f_$v -o run --output-format csv \
    -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-extras > $O/f_$v.json 2> $O/f_$v.err \
    || { tail -20 $O/f_$v.err; exit 1; }
  python3 - $O/f_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
v = [float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'ecmult_k4' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE']
print(sys.argv[2], 'k4 FETCH_SIZE KB per launch (raw, x2 for gfx950)', [round(x) for x in v[-3:]])
PY
done
