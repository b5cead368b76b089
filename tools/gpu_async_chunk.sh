# Submitted host batches: async_probe.py at several GV_ASYNC_CHUNK sizes (§5.1).
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/async_chunk}
mkdir -p $OUT
for c in ${CHUNKS:-262144 1048576 524288 786432 1048576 262144}; do
  echo "== chunk $c" >> $OUT/probe.jsonl
  GV_ASYNC_CHUNK=$c timeout -k 10 240 python3 tools/async_probe.py 1000000 6 >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done
grep -E "chunk|async" $OUT/probe.jsonl
