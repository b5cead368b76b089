set -o pipefail
for rep in 1 2; do
for cfg in "GV_HOST_LADDER_STREAM=1 GV_ASYNC_CHUNK=262144 GV_ASYNC_GROWTH=1" "GV_HOST_LADDER_STREAM=0 GV_ASYNC_CHUNK=262144 GV_ASYNC_GROWTH=1" "GV_HOST_LADDER_STREAM=0 GV_ASYNC_CHUNK=262144 GV_ASYNC_GROWTH=4" "GV_HOST_LADDER_STREAM=1 GV_ASYNC_CHUNK=131072 GV_ASYNC_GROWTH=1"; do
  echo "CFG $cfg" >> gpurun_out/async_ab.jsonl
  env $cfg timeout -k 10 300 python -u tools/async_probe.py 1000000 6 >> gpurun_out/async_ab.jsonl 2>> gpurun_out/async_ab.err || exit 1
done; done
