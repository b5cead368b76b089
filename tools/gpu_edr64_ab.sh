#!/bin/bash
# ed25519 grouped key tables as radix-64 combs (GV_ED_GROUP_R64 1, default)
# against radix-16: the ed25519 GPU tests, then the ed25519 bench line
# alternated, each run in a process of its own.
set -o pipefail
O=gpurun_out/edr64; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_ed_keyed_gpu.py tests/test_ed_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    GV_ED_GROUP_R64=$v timeout -k 10 240 python -u tools/ed_probe.py 1000000 16 > $O/r64_${v}_$i.json 2> $O/r64_${v}_$i.err || { tail -20 $O/r64_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/r64_${v}_$i.json'))
print('r64=$v run $i: grouped', round(d['value']/1e6,1), 'M/s kernel_ms', d.get('kernel_ms'), 'mism', d['mismatches'])"
  done
done
