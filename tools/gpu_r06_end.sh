#!/bin/bash
# Round 6 end: the default bench + its rocprofv3 kernel trace (gpu_end_round.sh
# bench), then the PMC passes over the resident arena's kw ladder at HEAD
# (the round-5 kw PMC predated the 64-B canonical entries).
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/r06_end}
bash tools/gpu_end_round.sh $OUT bench || exit 1
MODE=kw bash tools/pmc_round.sh $OUT/kw_pmc 1000000 || exit 1
python3 tools/pmc_summary.py $OUT/kw_pmc 1000000 $OUT/kw_pmc/pmc_summary.json > $OUT/kw_pmc/pmc_summary.txt 2>&1
tail -4 $OUT/kw_pmc/pmc_summary.txt
