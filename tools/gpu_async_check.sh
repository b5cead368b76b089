# Async host batches after a queue/chunking change: their tests, then the
# probe (sync / submitted, pageable / pinned) at the default chunking.
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/async_check}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_async.py tests/test_group_keys.py tests/test_multi_device.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python3 tools/async_probe.py 1000000 6 > $OUT/probe.jsonl 2> $OUT/probe.err || exit 1
timeout -k 10 240 python3 tools/async_probe.py 1000000 12 > $OUT/probe12.jsonl 2>> $OUT/probe.err || exit 1
cat $OUT/probe.jsonl $OUT/probe12.jsonl
