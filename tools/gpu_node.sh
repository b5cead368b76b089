set -o pipefail
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_block_paths.py tests/test_gas_order.py tests/test_ante_mirror.py tests/test_ibc_commits.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u tools/node_probe.py both 16 > $OUT/node.json 2> $OUT/node.err || { tail -30 $OUT/node.err; exit 1; }
cat $OUT/node.json
