set -o pipefail
OUT=gpurun_out/${1:-ed}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ed_keyed_gpu.py tests/test_ed_gpu.py tests/test_abi.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -30 $OUT/tests.log
exit $rc
