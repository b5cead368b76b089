# Keyed small batches on the wide arena's one-window tables
# (k_verify_lat16_kw, GV_LAT_KW=1) vs the kn tables (0): the keyed tests,
# then the bench's C5 curve (keyed p50 per batch size), alternated.
set -o pipefail
cd /root/repo
O=${1:-gpurun_out/latkw}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_key_cache.py tests/test_ladder_variants.py tests/test_gpu_parity.py tests/test_async.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    GV_LAT_KW=$v timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$i.json')); print('lat_kw $v rep $i', {k: v.get('keyed_p50_ms') for k, v in d['checktx_latency_ms'].items()})"
  done
done
