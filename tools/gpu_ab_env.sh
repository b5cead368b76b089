#!/bin/bash
# A/B of runtime settings on ONE box: bench.py (C2, no extras) per variant,
# alternated, REPS rounds.  Usage: tools/gpu_ab_env.sh OUT REPS "name:ENV=V ENV2=W" ...
set -o pipefail
cd /root/repo
OUT=$1; REPS=$2; shift 2
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --no-latency \
      > $OUT/b_${name}_$rep.json 2>>$OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "import json; b=json.load(open('$OUT/b_${name}_$rep.json')); p=b['pipeline']; print('$name', $rep, round(b['value']/1e6,2), 'step', b['ms_per_step'], 'ladder', p['ecmult_ms'], 'front', p['unpack_ms'], p['scalar_inv_ms'], p['prep_ms'], 'overl', p['pipelined_overlapped_stage_ms'], 'par', b['parity']['mismatches'], b['parity']['adversarial_mismatches'])"
  done
done
