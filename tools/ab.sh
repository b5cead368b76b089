#!/bin/bash
# A/B of library variants on ONE box (box-to-box clock spread is up to ~8 %):
# bench.py (C2, 1M, no extras) and the CheckTx curve for each library, twice,
# alternating.  Usage: tools/ab.sh OUT lib_a.so lib_b.so
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    GV_LIB="$lib" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline \
      > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { echo "bench $name failed"; tail -20 "$OUT/${name}_$rep.err"; exit 1; }
    python3 -c "import json,sys; b=json.load(open('$OUT/${name}_$rep.json')); print('$name', $rep, round(b['value']/1e6,2), 'M/s', b['pipeline'], 'p50@64', b['checktx_p50_ms_64'])"
  done
done
