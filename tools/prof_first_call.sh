# HIP API + kernel timeline of the first calls on a fresh context.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_first}
mkdir -p $OUT
timeout -k 10 300 python3 tools/first_call_probe.py 1000000 6 > $OUT/plain.json 2> $OUT/plain.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT -o run -- python3 tools/first_call_probe.py 1000000 6 > $OUT/probe.json 2> $OUT/probe.err || exit 1
cat $OUT/plain.json $OUT/probe.json
