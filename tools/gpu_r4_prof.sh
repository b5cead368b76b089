#!/bin/bash
# round 4: the PMC passes (tools/pmc_round.sh) over the headline bench command
set -o pipefail
cd /root/repo
O=gpurun_out/r4prof; mkdir -p $O
bash tools/pmc_round.sh $O/pmc 1000000 || exit 1
python3 tools/pmc_summary.py $O/pmc 1000000 $O/pmc_summary.json > $O/pmc_summary.txt 2>&1
tail -3 $O/pmc_summary.txt
