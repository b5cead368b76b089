#!/bin/bash
set -o pipefail
OUT=gpurun_out/v18
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
L=cosmos-sdk-rootchain_amd/lib
GV_LIB=$L/libgpuverify_trace.so timeout -k 10 200 python tools/lat_trace.py > "$OUT/lat_trace.json" 2> "$OUT/lat_trace.err" || { echo "trace failed"; tail -20 "$OUT/lat_trace.err"; exit 1; }
cat "$OUT/lat_trace.json"
timeout -k 10 300 python tools/lat_probe.py > "$OUT/lat_probe.json" 2> "$OUT/lat_probe.err" || { echo "probe failed"; tail -20 "$OUT/lat_probe.err"; exit 1; }
cat "$OUT/lat_probe.json"
GV_LIB=$L/libgpuverify_nosplit.so timeout -k 10 300 python tools/lat_probe.py > "$OUT/lat_probe_nosplit.json" 2> "$OUT/lat_probe2.err" || { echo "probe2 failed"; tail -20 "$OUT/lat_probe2.err"; exit 1; }
cat "$OUT/lat_probe_nosplit.json"
