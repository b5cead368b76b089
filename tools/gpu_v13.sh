#!/bin/bash
set -o pipefail
OUT=gpurun_out/v13
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_ante_mirror.py tests/test_key_cache.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python tools/lat_probe.py > "$OUT/lat_probe.json" 2> "$OUT/lat_probe.err" || { echo "probe failed"; tail -20 "$OUT/lat_probe.err"; exit 1; }
cat "$OUT/lat_probe.json"
