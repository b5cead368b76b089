#!/bin/bash
# Wide-window arena: its parity tests (ladder variants, HBM budget, key cache,
# async keyed batches), then the c2_key_cache A/B against the k6 tables.
set -o pipefail
O=gpurun_out/kw; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ladder_variants.py tests/test_hbm_budget.py tests/test_key_cache.py tests/test_async.py -x -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -8 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/kw_ab.py 2 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cut -c1-220 $O/ab.jsonl
