"""Secondary measurements reported inside bench.py's JSON line (rank 0, N=1).

  c2_key_cache    the C2 batch verified by account-key slot (gv_keys_load once,
                  then gv_dev_verify_digests_keyed): SURVEY.md §8f-2.
  c2_unique_keys  the C2 variant with one distinct key per item.
  c3_adversarial  BASELINE.json configs[2]: 1M signatures, 25 % invalid (high-S,
                  r >= n, s = 0 / 2^256-1, random x, malformed prefix, wrong
                  message), device-resident, bitmap checked against the verdicts
                  known by construction.
  msg_path        the full VerifyBytes path on MsgSend StdSignBytes (C1 message
                  shape, ~350-byte messages: SHA-256 on the GPU, one message per
                  lane) through gv_dev_verify_msgs, device-resident.
  c1_ante         BASELINE.json configs[0] shape: 10k single-signer MsgSend txs
                  through the host mirror of the ante chain (libgvhost) --
                  block path (PreVerifyTxs: one GPU batch, then the decorators
                  with verdict-cache hits) and the per-tx CheckTx path (one GPU
                  call per tx), host buffers / PCIe included.
  c4_multisig     BASELINE.json configs[3] shape on one GPU: k-of-n multisig
                  MsgSend txs replayed in blocks through PreVerifyTxs + ante.

Nothing here touches oracle/: verdicts come from construction (the workload
signs valid items with OpenSSL and mutates the invalid ones).
"""
from __future__ import annotations

import ctypes
import os
import struct
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))


def _unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]


def _timed_device_runs(ver, run, steps: int, warmup: int = 1):
    for _ in range(warmup):
        run()
    ver.dev_sync()
    ver.set_option("time_kernels", 1)
    ver.stage_stats()
    t = time.perf_counter()
    for _ in range(steps):
        run()
    ver.dev_sync()
    el = time.perf_counter() - t
    cnt, unpack_ms, prep_ms, ecmult_ms = ver.stage_stats()
    ver.set_option("time_kernels", 0)
    return el, {"unpack_or_sha_ms": round(unpack_ms, 3), "prep_ms": round(prep_ms, 3), "ecmult_ms": round(ecmult_ms, 3)}


def c2_unique_keys(ver, make_workload, n: int, threads: int, steps: int = 3):
    """SURVEY.md §8d C2 variant: one distinct key per item (no key reuse at
    all), device-resident, bitmap checked against construction."""
    pub, sig, dig, exp = make_workload(n, 0xC2 ^ 0x5A5A, n, 0.0, threads)
    d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
    for p, a in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, a)
    nw = (n + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    el, stages = _timed_device_runs(ver, lambda: ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits), steps)
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    got = _unpack_bits(bits, n)
    for p in d + [d_bits]:
        ver.dev_free(p)
    return {"items": n, "keys": n, "value": round(n * steps / el, 1), "unit": "verifies/s",
            "mismatches": int(np.count_nonzero(got != exp)), "stages": stages}


def c3_adversarial(ver, make_workload, n: int, threads: int, steps: int = 3):
    pub, sig, dig, exp = make_workload(n, 0xC3, 65536, 0.25, threads)
    d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
    for p, a in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, a)
    nw = (n + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    el, stages = _timed_device_runs(ver, lambda: ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits), steps)
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    got = _unpack_bits(bits, n)
    out = {"items": n, "invalid_fraction": round(1 - float(exp.mean()), 4),
           "value": round(n * steps / el, 1), "unit": "verifies/s",
           "mismatches": int(np.count_nonzero(got != exp)), "accepted": int(got.sum()),
           "expected_accepted": int(exp.sum()), "stages": stages}
    for p in d + [d_bits]:
        ver.dev_free(p)
    return out


def c2_key_cache(ver, pub, sig, dig, exp, nkeys: int, steps: int = 5):
    """SURVEY.md §8f-2 on the C2 batch: the 65,536 account keys are parsed once
    into the device key arena (gv_keys_load, timed on its own), then the same
    1M items are verified by slot (gv_dev_verify_digests_keyed, device
    resident): no per-item decompression or Q-table build.  Reported beside
    `value`, never as it (key parsing is hoisted out of the timed region)."""
    n = len(pub)
    ver.keys_reset()
    t = time.perf_counter()
    slots_k = ver.keys_load(pub[:nkeys])          # item i uses key i % nkeys (bench workload)
    t_load = time.perf_counter() - t
    slots = np.ascontiguousarray(slots_k[np.arange(n) % nkeys])
    d = [ver.dev_alloc(a.nbytes) for a in (slots, sig, dig)]
    for p, a in zip(d, (slots, sig, dig)):
        ver.dev_upload(p, a)
    nw = (n + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    el, stages = _timed_device_runs(ver, lambda: ver.dev_verify_digests_keyed(0, n, d[0], d[1], d[2], d_bits), steps)
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    got = _unpack_bits(bits, n)
    for p in d + [d_bits]:
        ver.dev_free(p)
    ver.keys_reset()
    return {"items": n, "keys": nkeys, "value": round(n * steps / el, 1), "unit": "verifies/s",
            "keys_load_ms": round(t_load * 1e3, 2), "mismatches": int(np.count_nonzero(got != exp)),
            "stages": stages,
            "note": "keys parsed once into the HBM key arena (1,280 B per key); items verified by slot"}


def c1_items(wl, n: int, threads: int, nkeys: int = 10000):
    """C1 item set: n MsgSend StdSignBytes messages for nkeys
    accounts (key i = GenPrivKeySecp256k1 over a C1 secret, account number i,
    sequence 0), signed with OpenSSL.  Returns pub, sig, (blob, off, len), and
    the expected verdicts (all valid)."""
    priv = np.zeros((nkeys, 32), np.uint8)
    pubk = np.zeros((nkeys, 33), np.uint8)
    wl.gvw_keys(nkeys, 0xC1, priv.ctypes.data, pubk.ctypes.data, threads)
    cap = n * 512
    blob = np.zeros(cap, np.uint8)
    off = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    wl.gvw_msgsend_signbytes.restype = ctypes.c_longlong
    wl.gvw_msgsend_signbytes.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    wl.gvw_sha256_msgs.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    total = wl.gvw_msgsend_signbytes(n, pubk.ctypes.data, nkeys, 0, blob.ctypes.data, cap, off.ctypes.data,
                                     ln.ctypes.data)
    assert total > 0
    blob = blob[:total].copy()
    mdig = np.zeros((n, 32), np.uint8)
    wl.gvw_sha256_msgs(n, blob.ctypes.data, off.ctypes.data, ln.ctypes.data, mdig.ctypes.data)
    pub = np.zeros((n, 33), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    dig = np.zeros((n, 32), np.uint8)
    exp = np.zeros(n, np.uint8)
    wl.gvw_sign(n, 0xC1, nkeys, priv.ctypes.data, pubk.ctypes.data, None, mdig.ctypes.data, 0.0,
                pub.ctypes.data, sig.ctypes.data, dig.ctypes.data, exp.ctypes.data, threads)
    return pub, sig, (blob, off, ln), exp


def msg_path(ver, wl, n: int, threads: int, nkeys: int = 10000, steps: int = 3):
    """wl: tools/workload/libgvwork.so handle (bench.workload_lib())."""
    pub, sig, (blob, off, ln), exp = c1_items(wl, n, threads, nkeys)
    arrs = (pub, sig, blob, off, ln)
    d = [ver.dev_alloc(a.nbytes) for a in arrs]
    for p, a in zip(d, arrs):
        ver.dev_upload(p, a)
    nw = (n + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    el, stages = _timed_device_runs(
        ver, lambda: ver.dev_verify_msgs(0, n, d[0], d[1], d[2], d[3], d[4], d_bits), steps)
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    got = _unpack_bits(bits, n)
    out = {"items": n, "mean_msg_bytes": round(float(ln.mean()), 1), "value": round(n * steps / el, 1),
           "unit": "verifies/s (SHA-256 of StdSignBytes + ECDSA)", "mismatches": int(np.count_nonzero(got != exp)),
           "stages": stages}
    for p in d + [d_bits]:
        ver.dev_free(p)
    return out


def c1_ante(ver, ntx: int = 10000, per_tx_sample: int = 500):
    import gvhost
    import txkit as T
    keys = []
    for i in range(ntx + 1):
        priv = T.privkey_from_secret(b"gv-c1-" + struct.pack("<Q", i))
        pub33 = T.secp_pubkey(priv)
        amino = T.amino_secp(pub33)
        keys.append((priv, amino, T.address(amino)))
    fee = T.fee_json([(0, "stake")], 1000000)
    txs = []
    for i in range(ntx):
        priv, amino, addr = keys[i]
        msg = T.msg_send_json(addr, keys[i + 1][2], [(10, "foocoin")])
        sb = T.std_sign_bytes("gv-bench", i, 0, fee, [msg], "")
        txs.append(T.flat_tx([msg], fee, "", [addr], [(amino, T.secp_sign(priv, sb))]))

    def fresh_app():
        app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
        for i in range(ntx):
            app.set_account(keys[i][2], i, 0)
        return app

    # block path: PreVerifyTxs (one GPU batch) + the ante chain per tx
    app = fresh_app()
    t = time.perf_counter()
    rc, leaves = app.preverify(txs)
    t_pre = time.perf_counter() - t
    ok = 0
    hits = 0
    for tx in txs:
        rc_a, r = app.ante(tx)
        ok += rc_a == 0 and r["code"] == 0
        hits += r["cache_hits"]
    t_block = time.perf_counter() - t
    app.close()
    # per-tx path (CheckTx without batching): one GPU call per tx
    app = fresh_app()
    m = min(per_tx_sample, ntx)
    t = time.perf_counter()
    ok2 = 0
    for tx in txs[:m]:
        rc_a, r = app.ante(tx)
        ok2 += rc_a == 0 and r["code"] == 0
    t_single = time.perf_counter() - t
    app.close()
    return {"txs": ntx, "block_path": {"txs_per_s": round(ntx / t_block, 1), "total_ms": round(t_block * 1e3, 2),
                                       "preverify_ms": round(t_pre * 1e3, 2), "accepted": ok, "cache_hits": hits,
                                       "gpu_leaves": leaves},
            "per_tx_path": {"txs": m, "txs_per_s": round(m / t_single, 1), "accepted": ok2},
            "note": "host mirror (libgvhost) of SetPubKey/ValidateSigCount/SigGasConsume/BatchSigVerification/"
                    "IncrementSequence over libgpuverify; sign bytes rebuilt per tx in C++; host buffers"}


def c4_multisig(ver, wl=None, ntx: int = 30000, block: int = 10000, naccounts: int = 96, threads: int = 16):
    """BASELINE.json configs[3] shape on one GPU: k-of-n threshold multisig
    MsgSend txs (2-of-3, 3-of-5, 4-of-7 in equal shares), replayed in blocks of
    `block` txs: gvh_preverify (every secp256k1 leaf of the block in one GPU
    batch, sequences predicted per signer) then the ante chain per tx.
    wl: tools/workload/libgvwork.so handle (batch signing with OpenSSL)."""
    import hashlib
    import gvhost
    import txkit as T
    shapes = [(2, 3), (3, 5), (4, 7)]
    privs, accts = [], []
    for a in range(naccounts):
        k, nsub = shapes[a % 3]
        base = len(privs)
        amino = []
        for j in range(nsub):
            priv = T.privkey_from_secret(b"gv-c4-" + struct.pack("<QQ", a, j))
            privs.append(priv)
            amino.append(T.amino_secp(T.secp_pubkey(priv)))
        mk = T.amino_multisig(k, amino)
        accts.append((k, nsub, base, mk, T.address(mk)))
    sink = T.address(T.amino_secp(T.secp_pubkey(T.privkey_from_secret(b"gv-c4-sink"))))
    fee = T.fee_json([(0, "stake")], 1000000)
    msgs, kidx, digs = [], [], []
    for i in range(ntx):
        a = i % naccounts
        k, nsub, base, mk, addr = accts[a]
        msg = T.msg_send_json(addr, sink, [(1, "foocoin")])
        sb = T.std_sign_bytes("gv-bench", a, i // naccounts, fee, [msg], "")
        msgs.append(msg)
        d = hashlib.sha256(sb).digest()
        for j in range(k):
            kidx.append(base + j)
            digs.append(d)
    L = len(kidx)
    priv_arr = np.frombuffer(b"".join(privs), np.uint8).reshape(-1, 32).copy()
    pub_arr = np.zeros((len(privs), 33), np.uint8)          # unused by gvw_sign's signing
    kid = np.array(kidx, np.uint32)
    dig = np.frombuffer(b"".join(digs), np.uint8).reshape(L, 32).copy()
    o_pub = np.zeros((L, 33), np.uint8)
    o_sig = np.zeros((L, 64), np.uint8)
    o_dig = np.zeros((L, 32), np.uint8)
    exp = np.zeros(L, np.uint8)
    wl.gvw_sign(L, 0xC4, len(privs), priv_arr.ctypes.data, pub_arr.ctypes.data, kid.ctypes.data, dig.ctypes.data,
                0.0, o_pub.ctypes.data, o_sig.ctypes.data, o_dig.ctypes.data, exp.ctypes.data, threads)
    txs, pos = [], 0
    for i in range(ntx):
        k, nsub, base, mk, addr = accts[i % naccounts]
        sigs = [o_sig[pos + j].tobytes() for j in range(k)]
        pos += k
        bits = [j < k for j in range(nsub)]
        txs.append(T.flat_tx([msgs[i]], fee, "", [addr], [(mk, T.multisignature(bits, sigs))]))
    app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
    for a, acct in enumerate(accts):
        app.set_account(acct[4], a, 0)
    ok = 0
    t_pre = 0.0
    t = time.perf_counter()
    for b0 in range(0, ntx, block):
        blk = txs[b0:b0 + block]
        tp = time.perf_counter()
        app.preverify(blk)
        t_pre += time.perf_counter() - tp
        for tx in blk:
            rc_a, r = app.ante(tx)
            ok += rc_a == 0 and r["code"] == 0
    el = time.perf_counter() - t
    app.close()
    return {"txs": ntx, "leaves": L, "block_txs": block, "accepted": ok,
            "leaves_per_s": round(L / el, 1), "txs_per_s": round(ntx / el, 1),
            "preverify_ms_per_block": round(t_pre * 1e3 / ((ntx + block - 1) // block), 2),
            "note": "2-of-3 / 3-of-5 / 4-of-7 threshold accounts, all k bits set; host mirror path with host buffers"}
