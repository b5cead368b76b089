#!/bin/bash
set -o pipefail
OUT=gpurun_out/v14
mkdir -p "$OUT"
GVH_PROFILE=1 timeout -k 10 120 python tools/host_probe.py > "$OUT/host_probe.txt" 2>&1 || { echo "host probe failed"; tail "$OUT/host_probe.txt"; exit 1; }
cat "$OUT/host_probe.txt"
timeout -k 10 300 python -u -m pytest tests/test_key_cache.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python tools/lat_probe.py > "$OUT/lat_probe.json" 2> "$OUT/lat_probe.err" || { echo "probe failed"; tail -20 "$OUT/lat_probe.err"; exit 1; }
cat "$OUT/lat_probe.json"
