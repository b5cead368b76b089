#!/bin/bash
# Round-4 GPU pass A: full GPU suite, then k6 (3 / 4 waves) vs k4 bench A/B,
# then a kernel trace of the pipelined k6 bench (overlap timeline).
set -o pipefail
cd /root/repo
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=cosmos-sdk-rootchain_amd/lib
for rep in 1 2; do
  for v in base k4 w4; do
    lib=$L/libgpuverify.so; env=""
    [ $v = w4 ] && lib=$L/libgpuverify_w4.so
    [ $v = k4 ] && env="GV_K6=0"
    env $env GV_LIB=$lib timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline \
      --no-latency > $O/b_${v}_$rep.json 2>>$O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; b=json.load(open('$O/b_${v}_$rep.json')); p=b['pipeline']; print('$v', $rep, round(b['value']/1e6,2), 'step', b['ms_per_step'], 'ladder', p['ecmult_ms'], 'front', p['unpack_ms'], p['scalar_inv_ms'], p['prep_ms'], 'overl', p['pipelined_overlapped_stage_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$O/trace -o k6 -- \
  python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency > /root/repo/$O/trace_bench.json 2>/root/repo/$O/trace.err \
  || { tail -20 /root/repo/$O/trace.err; exit 1; }
find /root/repo/$O/trace -name "*.csv" | head
