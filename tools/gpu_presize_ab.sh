# First calls on a fresh context with gv_open's pre-sizing (GV_PRESIZE=1) and
# without, alternated (tools/first_call_probe.py).
set -o pipefail
cd /root/repo
OUT=${1:-gpurun_out/presize}
mkdir -p $OUT
for rep in 1 2 3; do
  for w in 1 0; do
    echo "== presize $w" >> $OUT/probe.jsonl
    GV_PRESIZE=$w timeout -k 10 300 python3 tools/first_call_probe.py 1000000 6 >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
  done
done
python3 - $OUT/probe.jsonl <<'PY'
import json, sys
tag = None
for line in open(sys.argv[1]):
    if line.startswith("=="): tag = line.strip(); continue
    d = json.loads(line)
    print(tag, d["open_ms"], d["first_over_steady"], d["calls_ms"])
PY
