set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_group_keys.py tests/test_sort_keys.py > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
i=0
for k in 1 0 1 0; do
  i=$((i+1))
  GV_K6=$k timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency > gpurun_out/b1_k6_${k}_$i.json 2>>gpurun_out/b1.err || { tail -20 gpurun_out/b1.err; exit 1; }
  python3 -c "import json; b=json.load(open('gpurun_out/b1_k6_${k}_$i.json')); print('k6=$k', round(b['value']/1e6,2), b['ms_per_step'], b.get('roofline',{}).get('frac'), b.get('parity'))"
done
