# Kernel + copy timeline of the host-buffer paths (tools/async_probe.py:
# synchronous and submitted batches, pageable and pinned) for §5.1.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_async}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace ${EXTRA_TRACE:-} --output-format csv -d $OUT -o run -- python3 tools/async_probe.py 1000000 6 > $OUT/probe.jsonl 2> $OUT/probe.err || exit 1
cat $OUT/probe.jsonl
