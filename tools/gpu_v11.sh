#!/bin/bash
# v11: GPU tests + bench + kernel trace of the default build, then a same-box
# A/B of the doubling / occupancy variants.
set -o pipefail
bash tools/gpu_round.sh gpurun_out/v11 || exit 1
bash tools/ab.sh gpurun_out/v11/ab cosmos-sdk-rootchain_amd/lib/libgpuverify.so \
  cosmos-sdk-rootchain_amd/lib/libgpuverify_dbl25.so cosmos-sdk-rootchain_amd/lib/libgpuverify_occ4.so \
  cosmos-sdk-rootchain_amd/lib/libgpuverify_noilp.so
