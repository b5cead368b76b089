import os, sys, json
sys.path.insert(0, "."); sys.path.insert(0, "cosmos-sdk-rootchain_amd"); sys.path.insert(0, "tools")
import bench, bench_extras as X, gpuverify as gvm
ver = gvm.Verifier([0])
r = X.c1_ante(ver, wl=bench.workload_lib(), threads=16)
print(json.dumps({k: r[k] for k in ("block_path_steady", "block_path")}))
