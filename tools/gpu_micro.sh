#!/bin/bash
# GPU-box microbenchmarks of the field layers (each step time-limited; the
# chain stops at the first failure).
set -o pipefail
OUT=${1:-gpurun_out/micro}
mkdir -p "$OUT"
for b in "${@:2}"; do
  echo "== $b" | tee -a "$OUT/micro.log"
  timeout -k 10 120 "$b" >> "$OUT/micro.log" 2>&1 || { echo "$b failed"; tail -20 "$OUT/micro.log"; exit 1; }
done
cat "$OUT/micro.log"
