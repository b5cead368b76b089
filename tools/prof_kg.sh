set -o pipefail
cd /root/repo
export TMPDIR=/tmp
for v in 0 9; do
  GV_KG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kg$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --no-latency > gpurun_out/prof_kg$v.json 2> gpurun_out/prof_kg$v.err || exit 1
done
