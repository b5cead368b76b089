#!/bin/bash
# GPU tests -> bench (with extras) -> 10M-signature parity.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/full}
M=${2:-10}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" && mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ "$M" -gt 0 ]; then
  GV_PARITY_MILLIONS=$M GV_PARITY_OUT="$OUT/parity.json" timeout -k 10 900 python -m pytest tests/test_parity_large.py -q -s -p no:cacheprovider > "$OUT/parity.log" 2>&1 || { echo "parity failed"; tail -30 "$OUT/parity.log"; exit 1; }
  tail -3 "$OUT/parity.log"
fi
