# Round end at HEAD: the whole GPU suite, smoke(), then the default bench line.
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/final3}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 200 $OUT/bench.json
