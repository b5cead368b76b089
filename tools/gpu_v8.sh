set -o pipefail
mkdir -p gpurun_out/v8
timeout -k 10 120 tools/microbench/fe29_rate lat > gpurun_out/v8/lat.log 2>&1 && cat gpurun_out/v8/lat.log &&
bash tools/gpu_round.sh gpurun_out/v8
