#!/bin/bash
# Block replay through the host mirror with block b+1's batch queued on the
# asynchronous entry points (GVH_ASYNC_BLOCKS=1, default) vs on a helper
# thread's synchronous call (0), alternated; C1 + C4 node lines per run.
set -o pipefail
out=${1:-gpurun_out/async_blocks_ab.jsonl}
: > "$out"
for rep in 0 1; do
  for a in 1 0; do
    echo "{\"GVH_ASYNC_BLOCKS\": $a, \"rep\": $rep}" >> "$out"
    GVH_ASYNC_BLOCKS=$a timeout -k 10 240 python -u tools/node_probe.py both 16 >> "$out" 2>/dev/null || exit 1
  done
done
