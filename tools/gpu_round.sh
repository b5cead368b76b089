#!/bin/bash
# One GPU-box session.  Steps (each with its own time limit; the chain stops
# at the first failure):
#   tests   pytest -m gpu (per-test timeout, thread method)
#   bench   python bench.py (headline line + extras)
#   prof    rocprofv3 --kernel-trace --stats over the headline bench command
#   profed  the same over tools/ed_probe.py (ed25519 throughput + cached-key small batches)
#   parity  tests/test_parity_large.py at M million signatures (M > 0)
# usage: tools/gpu_round.sh OUT "tests bench prof parity" [M]
set -o pipefail
OUT=${1:-gpurun_out/run}
STEPS=${2:-"tests bench prof"}
M=${3:-10}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" && mkdir -p "$OUT"
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -60 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
if has bench; then
  timeout -k 10 1000 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
if has prof; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-extras \
      > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/bench_prof.err" ) || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
  python3 tools/prof_timed.py "$OUT/prof/run_kernel_trace.csv" 5 "$OUT/prof/kernel_timed.csv"
fi
if has profed; then                      # the ed25519 kernels incl. the cached-key small-batch kernel
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/profed" -o run \
      --output-format csv -- python3 "$ROOT/tools/ed_probe.py" 200000 16 \
      > "$ROOT/$OUT/ed_prof.json" 2> "$ROOT/$OUT/ed_prof.err" ) || { echo "rocprof ed failed"; tail -30 "$OUT/ed_prof.err"; exit 1; }
fi
if has parity && [ "$M" -gt 0 ]; then
  GV_PARITY_MILLIONS=$M GV_PARITY_OUT="$OUT/parity.json" timeout -k 10 1000 python -u -m pytest tests/test_parity_large.py \
    -q -s -p no:cacheprovider > "$OUT/parity.log" 2>&1 || { echo "parity failed"; tail -30 "$OUT/parity.log"; exit 1; }
  tail -3 "$OUT/parity.log"
fi
echo done
