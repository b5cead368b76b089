#!/bin/bash
# Round 6 A/B: key-table back-propagation prefetch (GV_KEYS_PREFETCH), the
# quad table kernel at 4 waves/SIMD (GV_KEYS_TABLES_W4), on k4 and kg layouts.
L=cosmos-sdk-rootchain_amd/lib
exec bash tools/gpu_ab_env.sh gpurun_out/pf_ab 2 k4:GV_KG=0 kg9:GV_KG=9 kg7:GV_KG=7 \
  "k4_nopf:GV_LIB=$L/libgpuverify_nopf.so GV_KG=0" "kg9_nopf:GV_LIB=$L/libgpuverify_nopf.so GV_KG=9" \
  "k4_pf3:GV_LIB=$L/libgpuverify_pf3.so GV_KG=0"
