"""A/B of host-mirror settings given as environment variables read when an
app is created (GVH_GPU_HASH, GVH_DEFER_RELEASE, ...): C1 steady blocks (10k
single-signer txs, one block at a time and as one pipelined replay) and a C4
multisig replay (one block at a time and pipelined), settings alternated on
one box.  Prints one JSON line per (rep, setting).
usage: mirror_ab.py reps c4_accounts c4_txs_per_account name:VAR=V[,VAR=V] name:...
(the first round-4 use, the gpu_hash A/B, passed no settings: gpu_hash on/off)"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402
import gvhost  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
na = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
per = int(sys.argv[3]) if len(sys.argv) > 3 else 12
settings = []
for a in sys.argv[4:]:
    name, kv = a.split(":", 1)
    settings.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
if not settings:
    settings = [("gpu_hash", {"GVH_GPU_HASH": "1"}), ("host_hash", {"GVH_GPU_HASH": "0"})]
wl = bench.workload_lib()
ver = gvm.Verifier([0])
ntx = 10000
W = X.c1_blocks(wl, ntx, 8, 16)
later = W["later_blobs"]
cat = np.concatenate([b[0] for b in later])
base = np.cumsum([0] + [len(b[0]) for b in later[:-1]]).astype(np.uint64)
offs1 = np.concatenate([b[1] + base[k] for k, b in enumerate(later)])
lens1 = np.concatenate([b[2] for b in later])
blob4, offs4, lens4, accts4, leaves4 = X.c4_workload(wl, na, per, 16)
n4 = len(offs4)
nb4 = (n4 + 9999) // 10000


def c1_app():
    app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
    app.set_threads(16)
    for i in range(ntx):
        app.set_account(W["keys"][i][2], i, 0)
    rc, _ = app.deliver_block_blob(*W["first_blob"])
    assert rc == 0
    return app


def c1():
    app = c1_app()
    t = time.perf_counter()
    for b in later:
        rc, c = app.deliver_block_blob(*b)
        assert rc == 0 and (c == 0).all()
    one = ntx * len(later) / (time.perf_counter() - t)
    st = app.stats()
    app.close()
    app = c1_app()
    t = time.perf_counter()
    rc, cp = app.deliver_blocks_blob(cat, offs1, lens1, [len(b[1]) for b in later])
    piped = ntx * len(later) / (time.perf_counter() - t)
    app.close()
    assert rc == 0 and (cp == 0).all()
    return one, piped, st


def c4_app():
    app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
    app.set_threads(16)
    for addr, num in accts4:
        app.set_account(addr, num, 0)
    return app


def c4():
    app = c4_app()
    t = time.perf_counter()
    for b0 in range(0, n4, 10000):
        rc, codes = app.deliver_block_blob(blob4, offs4[b0:b0 + 10000], lens4[b0:b0 + 10000])
        assert rc == 0 and not np.count_nonzero(codes)
    one = leaves4 / (time.perf_counter() - t)
    app.close()
    app = c4_app()
    t = time.perf_counter()
    rc, codes = app.deliver_blocks_blob(blob4, offs4, lens4, [min(10000, n4 - b * 10000) for b in range(nb4)])
    el = time.perf_counter() - t
    st = app.stats()
    app.close()
    assert rc == 0 and not np.count_nonzero(codes)
    return one, leaves4 / el, st


def apply(env):
    for k, v in env.items():
        os.environ[k] = v


for name, env in settings:                                # warm-up
    apply(env)
    c1()
    c4()
for r in range(reps):
    for name, env in (settings if r % 2 == 0 else settings[::-1]):
        apply(env)
        one, piped, st1 = c1()
        one4, lps, st4 = c4()
        print(json.dumps({"rep": r, "name": name, "c1_one_block_txs_per_s": round(one), "c1_piped_txs_per_s": round(piped),
                          "c1_preverify_ms_per_block": round(st1["preverify_ns"] / 1e6 / (len(later) + 1), 3),
                          "c1_gpu_ms_per_block": round(st1["gpu_ns"] / 1e6 / (len(later) + 1), 3),
                          "c4_one_block_leaves_per_s": round(one4), "c4_leaves_per_s": round(lps), "c4_preverify_s": round(st4["preverify_ns"] / 1e9, 3),
                          "c4_gpu_s": round(st4["gpu_ns"] / 1e9, 3)}), flush=True)
ver.close()
