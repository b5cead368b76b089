set -o pipefail
OUT=gpurun_out/ed3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ed_keyed_gpu.py tests/test_ibc_commits.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E 'passed|failed|p50' $OUT/tests.log
timeout -k 10 300 python -u tools/ed_probe.py 1000000 16 > $OUT/ed.json 2> $OUT/ed.err || { tail -30 $OUT/ed.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/ed.json'));print(d['value'], json.dumps({k:(v['keyed_sliced_p50_ms'],v['throughput_p50_ms']) for k,v in d['small_batches']['batches'].items()}))"
timeout -k 10 300 python -u tools/hostpath_sweep.py 4 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -30 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
