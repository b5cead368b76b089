#!/bin/bash
# key-cache iteration: its GPU tests, then the full GPU suite, then the bench.
set -o pipefail
OUT=${1:-gpurun_out/keys}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_key_cache.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/key_tests.log" 2>&1 || { echo "key tests failed"; tail -40 "$OUT/key_tests.log"; exit 1; }
tail -3 "$OUT/key_tests.log"
bash tools/gpu_round.sh "$OUT"
