set -o pipefail
O=gpurun_out/item
mkdir -p $O
timeout -k 10 400 python3 -u tools/hostpath_probe.py > $O/hostpath_probe.jsonl 2> $O/hostpath_probe.err || { tail -20 $O/hostpath_probe.err; exit 1; }
cat $O/hostpath_probe.jsonl
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-extras --keys 1000000 > "$R/$O/bench_item.json" 2> "$R/$O/bench_item.err" ) || { tail -20 $O/bench_item.err; exit 1; }
python3 tools/prof_timed.py $O/prof/run_kernel_trace.csv 10 $O/prof/kernel_timed.csv > $O/prof/timed.txt && head -8 $O/prof/timed.txt
MODE=item bash tools/pmc_round.sh $O/pmc 1000000 || exit 1
python3 tools/pmc_summary.py $O/pmc 1000000 $O/pmc/pmc_summary.json > $O/pmc/pmc_summary.txt 2>&1; cat $O/pmc/pmc_summary.txt | grep -v gen_
