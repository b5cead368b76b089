#!/bin/bash
# A/B of in-batch key grouping on the headline bench (20 steps): GV_GROUP_KEYS=1 / 0 alternated.
OUT=${1:-gpurun_out/group_ab}; R=${2:-2}
mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for g in 1 0; do
    GV_GROUP_KEYS=$g timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-extras --no-latency --no-cpu-baseline \
      > "$OUT/g${g}_$r.json" 2> "$OUT/g${g}_$r.err" || { echo "bench failed g=$g"; tail -20 "$OUT/g${g}_$r.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/g${g}_$r.json')); print('group=$g', round(d['value']/1e6,2), 'M/s', d['pipeline']['serialized_sum_ms'], d['pipeline']['pipelined_ms_per_step'], 'frac', d['roofline']['frac'], 'mism', d['parity']['mismatches'], d['parity']['adversarial_mismatches'])"
  done
done
