#!/bin/bash
# One GPU-box session: GPU tests, bench, rocprofv3 kernel trace.  Each GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/run}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd "$ROOT"
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-extras --items 1000000 > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/bench_prof.err" || { echo "rocprof failed"; tail -30 "$ROOT/$OUT/bench_prof.err"; exit 1; }
find "$ROOT/$OUT/prof" -name "*stats*" | head
