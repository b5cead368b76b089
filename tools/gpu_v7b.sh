set -o pipefail
mkdir -p gpurun_out/v7b
timeout -k 10 120 tools/microbench/fe29_rate lat > gpurun_out/v7b/lat.log 2>&1 && cat gpurun_out/v7b/lat.log &&
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 -p no:cacheprovider > gpurun_out/v7b/gpu_tests.log 2>&1; tail -3 gpurun_out/v7b/gpu_tests.log
