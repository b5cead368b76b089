#!/bin/bash
# One iteration on the GPU box: tests + bench + rocprofv3 kernel stats, then
# (optional, PMC=1) the four PMC passes and their summary.  Each GPU step is
# time-limited and the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/iter}
bash tools/gpu_round.sh "$OUT" || exit 1
if [ "${PMC:-0}" = "1" ]; then
  bash tools/pmc_round.sh "$OUT/pmc" 1000000 || exit 1
  python3 tools/pmc_summary.py "$OUT/pmc" 1000000 "$OUT/pmc/summary.json" || exit 1
fi
