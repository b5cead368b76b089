#!/bin/bash
set -o pipefail
OUT=gpurun_out/v15
mkdir -p "$OUT"
GVH_PROFILE=1 timeout -k 10 120 python tools/host_probe.py > "$OUT/host_probe.txt" 2>&1 || { echo "host probe failed"; tail "$OUT/host_probe.txt"; exit 1; }
grep threads "$OUT/host_probe.txt"
timeout -k 10 200 python tools/lat_trace.py > "$OUT/lat_trace.json" 2> "$OUT/lat_trace.err" || { echo "trace failed"; tail -20 "$OUT/lat_trace.err"; exit 1; }
cat "$OUT/lat_trace.json"
