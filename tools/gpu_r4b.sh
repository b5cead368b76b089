#!/bin/bash
# Round-4 GPU pass B: grouped/sort/multi-stream tests, then the pipelining
# A/B (two ladder streams on/off, front kernels capped at 96 VGPRs), k4 for
# reference, and a kernel trace of the default build.
set -o pipefail
cd /root/repo
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_group_keys.py tests/test_sort_keys.py tests/test_multi_device.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=cosmos-sdk-rootchain_amd/lib
for rep in 1 2; do
  for v in base one f96 k4; do
    lib=$L/libgpuverify.so; env=""
    [ $v = f96 ] && lib=$L/libgpuverify_f96.so
    [ $v = one ] && env="GV_TWO_LADDERS=0"
    [ $v = k4 ] && env="GV_K6=0"
    env $env GV_LIB=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
      --no-latency > $O/b_${v}_$rep.json 2>>$O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; b=json.load(open('$O/b_${v}_$rep.json')); p=b['pipeline']; print('$v', $rep, round(b['value']/1e6,2), 'step', b['ms_per_step'], 'ladder', p['ecmult_ms'], 'front', p['unpack_ms'], p['scalar_inv_ms'], p['prep_ms'], 'overl', p['pipelined_overlapped_stage_ms'], 'par', b['parity']['mismatches'], b['parity']['adversarial_mismatches'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base f96; do
  lib=/root/repo/$L/libgpuverify.so; [ $v = f96 ] && lib=/root/repo/$L/libgpuverify_f96.so
  GV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$O/trace_$v -o t -- \
    python3 /root/repo/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-latency > /root/repo/$O/trace_$v.json 2>/root/repo/$O/trace_$v.err \
    || { tail -20 /root/repo/$O/trace_$v.err; exit 1; }
done
ls /root/repo/$O/trace_base
