#!/bin/bash
# ed25519 [s]B from the radix-2^16 comb table (GV_ED_BTAB16 1, default) against
# the radix-256 one: the keyed / grouped ed25519 GPU tests, then the ed25519
# bench line alternated, each run in a process of its own.
set -o pipefail
O=gpurun_out/ed16; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_ed_keyed_gpu.py tests/test_ed_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    GV_ED_BTAB16=$v timeout -k 10 240 python -u tools/ed_probe.py 1000000 16 > $O/b16_${v}_$i.json 2> $O/b16_${v}_$i.err || { tail -20 $O/b16_${v}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$O/b16_${v}_$i.json')); k=d.get('keyed_throughput',{}).get('keyed',{})
print('btab16=$v run $i: grouped', round(d['value']/1e6,1), 'M/s  keyed', round(k.get('value',0)/1e6,1), 'M/s  kernel_ms', d.get('kernel_ms'), 'mism', d['mismatches'])"
  done
done
