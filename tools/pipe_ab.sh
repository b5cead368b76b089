#!/bin/bash
# A/B of the pipelined device-resident path: bench.py headline (20 steps),
# GV_PIPELINE=1 / 0 alternated.  usage: tools/pipe_ab.sh OUT [rounds]
OUT=${1:-gpurun_out/pipe_ab}; R=${2:-2}
mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for p in 1 0; do
    GV_PIPELINE=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-extras --no-latency --no-cpu-baseline \
      > "$OUT/p${p}_$r.json" 2> "$OUT/p${p}_$r.err" || { echo "bench failed p=$p"; tail -20 "$OUT/p${p}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/p${p}_$r.json')); print('pipe=$p', round(d['value']/1e6,2), 'M/s', d['pipeline'], 'frac', d['roofline']['frac'], 'mism', d['parity']['mismatches'], d['parity']['adversarial_mismatches'])"
  done
done
