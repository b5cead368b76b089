set -o pipefail
OUT=gpurun_out/ed2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ibc_commits.py tests/test_ed_keyed_gpu.py tests/test_block_paths.py -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/ed_probe.py 1000000 16 > $OUT/ed.json 2> $OUT/ed.err || { tail -30 $OUT/ed.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/ed.json'));print(d['value'], json.dumps(d['small_batches']))"
