#!/bin/bash
# ed25519 option A/B: the ed25519 GPU tests, then the ed25519 bench line with
# the environment variable VAR at 1 and 0, alternated, each run in a process of
# its own (e.g. GV_ED_BTAB16, GV_ED_GROUP_R64).  usage: gpu_ed_ab.sh VAR [reps]
set -o pipefail
VAR=$1; R=${2:-2}
O=gpurun_out/ed_ab_$VAR; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_ed_keyed_gpu.py tests/test_ed_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
for i in $(seq 1 $R); do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 240 python -u tools/ed_probe.py 1000000 16 > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${v}_$i.json'))
print('$VAR=$v run $i: grouped', round(d['value']/1e6,1), 'M/s kernel_ms', d.get('kernel_ms'), 'mism', d['mismatches'])"
  done
done
