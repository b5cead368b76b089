#!/bin/bash
# A/B: key-table forward entries through coalesced scratch (GV_KEYS_SCRATCH=1)
# vs through the table (0), bench.py headline, alternated; then the keyed
# GPU tests.  usage: tools/ks_ab.sh OUT [rounds]
OUT=${1:-gpurun_out/ks_ab}; R=${2:-2}
mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for p in 1 0; do
    GV_KEYS_SCRATCH=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-extras --no-latency --no-cpu-baseline \
      > "$OUT/k${p}_$r.json" 2> "$OUT/k${p}_$r.err" || { echo "bench failed k=$p"; tail -20 "$OUT/k${p}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/k${p}_$r.json')); print('scratch=$p', round(d['value']/1e6,2), 'M/s', d['roofline']['kernels'], 'mism', d['parity']['mismatches'], d['parity']['adversarial_mismatches'])"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_group_keys.py tests/test_key_cache.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
