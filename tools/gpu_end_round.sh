#!/bin/bash
# End-of-round measurements on one GPU box, in two calls (each under gpurun's
# 20-minute limit); every GPU step has its own time limit and the chain stops
# at the first failure.
#   bench  the default bench (headline line + extras), then rocprofv3
#          --kernel-trace --stats over the headline bench command and the
#          per-kernel launch durations of its timed region
#   pmc    the GPU suite, then the PMC passes over the headline bench command
# usage: tools/gpu_end_round.sh OUT bench|pmc
set -o pipefail
OUT=${1:-gpurun_out/end}
WHAT=${2:-bench}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" && mkdir -p "$OUT"
if [ "$WHAT" = bench ]; then
  timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  tail -c 400 "$OUT/bench.json"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-extras \
      > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/bench_prof.err" ) || { tail -30 "$OUT/bench_prof.err"; exit 1; }
  python3 tools/prof_timed.py "$OUT/prof/run_kernel_trace.csv" 10 "$OUT/prof/kernel_timed.csv" > "$OUT/prof/timed.txt"
  head -12 "$OUT/prof/timed.txt"
else
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
  bash tools/pmc_round.sh "$OUT/pmc" 1000000 || exit 1
  python3 tools/pmc_summary.py "$OUT/pmc" 1000000 "$OUT/pmc/pmc_summary.json" > "$OUT/pmc/pmc_summary.txt" 2>&1
  tail -5 "$OUT/pmc/pmc_summary.txt"
fi
