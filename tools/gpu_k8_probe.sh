set -o pipefail
O=gpurun_out/k8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ladder_variants.py tests/test_hbm_budget.py -x -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread -k "cached or k8 or budget" > $O/tests.log 2>&1; rc=$?; tail -25 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/k8_ab.py 2 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cut -c1-220 $O/ab.jsonl
