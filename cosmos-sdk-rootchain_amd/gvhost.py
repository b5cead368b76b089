"""gvhost.py -- ctypes binding of libgvhost.so (host/gvhost.h), the C++ mirror
of the reference's signature-verification ante decorators over libgpuverify.

  HostApp.ante(tx)        SetPubKey -> ValidateSigCount -> SigGasConsume ->
                          BatchSigVerification -> IncrementSequence
                          (x/auth/ante/ante.go:13-31, sigverify.go) on an amino StdTx
  HostApp.preverify(txs)  block pre-verification hook
  HostApp.deliver_block   PreVerifyTxs + the DeliverTx ante loop (baseapp/abci.go:203-221)
  HostApp.deliver_gentxs  genutil.DeliverGenTxs (x/genutil/gentx.go:96-114)
  HostApp.checktx(tx)     CheckTx through the accumulation window (thread-safe)
"""
from __future__ import annotations

import ctypes
import os

import gpuverify as gvm

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GVH_LIB") or os.path.join(HERE, "lib", "libgvhost.so")  # GVH_LIB: A/B builds

GVH_OK, GVH_EINVAL, GVH_EDEVICE, GVH_ENOVERIFIER = 0, -1, -2, -3


class Result(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint32), ("codespace", ctypes.c_char * 16), ("log", ctypes.c_char * 512),
                ("gas_used", ctypes.c_uint64), ("gpu_leaves", ctypes.c_uint32), ("cache_hits", ctypes.c_uint32),
                ("gas_wanted", ctypes.c_uint64)]

    def as_dict(self):
        return {"code": self.code, "codespace": self.codespace.decode(), "log": self.log.decode(),
                "gas_used": self.gas_used, "gpu_leaves": self.gpu_leaves, "cache_hits": self.cache_hits,
                "gas_wanted": self.gas_wanted}


class Stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("gpu_calls", "gpu_leaves", "cache_hits", "cache_misses", "memo_hits",
                                               "windows", "window_txs", "cache_entries", "cache_capacity",
                                               "preverify_ns", "gpu_ns", "deliver_loop_ns")]


class Commit(ctypes.Structure):
    """gvh_commit (gvhost.h): one VerifyCommit / VerifyCommitTrusting check."""
    _fields_ = [("trusting", ctypes.c_int), ("trust_num", ctypes.c_int64), ("trust_den", ctypes.c_int64),
                ("basic_ok", ctypes.c_int), ("n_vals", ctypes.c_size_t), ("val_pub32", ctypes.c_void_p),
                ("val_addr20", ctypes.c_void_p), ("val_power", ctypes.c_void_p), ("n_sigs", ctypes.c_size_t),
                ("flag", ctypes.c_void_p), ("sig_addr20", ctypes.c_void_p), ("sig64", ctypes.c_void_p),
                ("sig_len", ctypes.c_void_p), ("msg_blob", ctypes.c_void_p), ("msg_off", ctypes.c_void_p),
                ("msg_len", ctypes.c_void_p), ("keys_trusted", ctypes.c_int)]


class CommitResult(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("idx", ctypes.c_int32), ("idx2", ctypes.c_int32),
                ("got", ctypes.c_int64), ("needed", ctypes.c_int64)]


COMMIT_CODES = {0: "ok", 1: "basic", 2: "size", 3: "wrong_sig", 4: "not_enough", 5: "double_vote", 6: "bad_trust"}

_L = None


def lib():
    global _L
    if _L is None:
        gvm.load()                       # libgvhost links libgpuverify
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t
        L.gvh_app_new.restype = vp
        L.gvh_app_new.argtypes = [vp]
        L.gvh_app_free.argtypes = [vp]
        L.gvh_set_params.argtypes = [vp, u64, u64, u64]
        L.gvh_set_gas_model.argtypes = [vp, ctypes.c_int]
        L.gvh_set_context.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, u64]
        L.gvh_set_account.argtypes = [vp, ctypes.c_char_p, u64, u64, ctypes.c_char_p, sz]
        L.gvh_get_account.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(u64), vp,
                                      ctypes.POINTER(sz)]
        L.gvh_ante.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_int, ctypes.POINTER(Result)]
        L.gvh_preverify.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.gvh_consume_sig_gas.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, sz, u64, ctypes.POINTER(Result)]
        L.gvh_cache_clear.argtypes = [vp]
        L.gvh_set_threads.argtypes = [vp, ctypes.c_int]
        L.gvh_set_keyed.argtypes = [vp, ctypes.c_int, ctypes.c_size_t]
        L.gvh_set_gpu_hash.argtypes = [vp, ctypes.c_int]
        L.gvh_get_gpu_hash.argtypes = [vp]
        L.gvh_get_keyed.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.gvh_cache_size.argtypes = [vp]
        L.gvh_cache_size.restype = sz
        L.gvh_std_sign_bytes.argtypes = [ctypes.c_char_p, u64, u64, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                         sz, ctypes.c_char_p, vp, sz]
        L.gvh_std_sign_bytes.restype = sz
        L.gvh_pubkey_address.argtypes = [ctypes.c_char_p, sz, vp]
        L.gvh_bech32_address.argtypes = [ctypes.c_char_p, vp, sz]
        L.gvh_bech32_address.restype = sz
        cpp = ctypes.POINTER(ctypes.c_char_p)
        L.gvh_deliver_block.argtypes = [vp, sz, cpp, ctypes.POINTER(sz), ctypes.POINTER(Result)]
        L.gvh_deliver_block_codes.argtypes = [vp, sz, cpp, ctypes.POINTER(sz), ctypes.POINTER(ctypes.c_uint32)]
        L.gvh_deliver_blocks.argtypes = [vp, sz, ctypes.POINTER(sz), cpp, ctypes.POINTER(sz),
                                         ctypes.POINTER(ctypes.c_uint32)]
        L.gvh_deliver_gentxs.argtypes = [vp, sz, cpp, ctypes.POINTER(sz), ctypes.POINTER(Result), ctypes.POINTER(sz)]
        L.gvh_checktx.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(Result)]
        L.gvh_set_window.argtypes = [vp, sz, ctypes.c_int64]
        L.gvh_set_cache_capacity.argtypes = [vp, sz]
        L.gvh_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
        L.gvh_tx_sign_bytes.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, u64, u64, vp, sz, vp, sz]
        L.gvh_verify_commits.argtypes = [vp, sz, ctypes.POINTER(Commit), ctypes.POINTER(CommitResult)]
        L.gvh_tx_sign_bytes.restype = sz
        _L = L
    return _L


def pubkey_address(pub_amino: bytes) -> bytes:
    out = ctypes.create_string_buffer(20)
    if lib().gvh_pubkey_address(pub_amino, len(pub_amino), out) != 0:
        raise ValueError("malformed amino pubkey")
    return out.raw


def bech32_address(addr20: bytes) -> str:
    out = ctypes.create_string_buffer(128)
    lib().gvh_bech32_address(addr20, out, 128)
    return out.value.decode()


def std_sign_bytes(chain_id: str, accnum: int, seq: int, fee_json: str, msgs_json, memo: str) -> bytes:
    arr = (ctypes.c_char_p * max(1, len(msgs_json)))(*[m.encode() for m in msgs_json])
    n = lib().gvh_std_sign_bytes(chain_id.encode(), accnum, seq, fee_json.encode(), arr, len(msgs_json),
                                 memo.encode(), None, 0)
    buf = ctypes.create_string_buffer(n)
    lib().gvh_std_sign_bytes(chain_id.encode(), accnum, seq, fee_json.encode(), arr, len(msgs_json), memo.encode(),
                             buf, n)
    return buf.raw


def tx_sign_bytes(tx: bytes, chain_id: str, accnum: int, seq: int) -> bytes:
    """DefaultTxDecoder + StdTx.GetSignBytes; raises ValueError(decode error) if the tx does not decode."""
    cap = 1 << 16
    out = ctypes.create_string_buffer(cap)
    err = ctypes.create_string_buffer(512)
    n = lib().gvh_tx_sign_bytes(tx, len(tx), chain_id.encode(), accnum, seq, out, cap, err, 512)
    if n == 0:
        raise ValueError(err.value.decode())
    return out.raw[:n]


def _arrays(txs):
    arr = (ctypes.c_char_p * max(1, len(txs)))(*txs)
    lens = (ctypes.c_size_t * max(1, len(txs)))(*[len(t) for t in txs])
    return arr, lens


class HostApp:
    def __init__(self, verifier: gvm.Verifier | None = None, chain_id: str = "gv-test", height: int = 1):
        self._L = lib()
        self._v = verifier
        self._app = self._L.gvh_app_new(verifier._ctx if verifier is not None else None)
        self.set_context(chain_id, height)

    def close(self):
        if self._app:
            self._L.gvh_app_free(self._app)
            self._app = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, tx_sig_limit=7, cost_secp=1000, cost_ed=590):
        self._L.gvh_set_params(self._app, tx_sig_limit, cost_secp, cost_ed)

    def set_gas_model(self, kv_gas: bool):
        """kv_gas: charge the ante chain's KV-store / params / tx-size gas (default) or signature gas only."""
        self._L.gvh_set_gas_model(self._app, int(kv_gas))

    def set_context(self, chain_id: str, height: int = 1, recheck: bool = False, gas_limit: int = 0):
        self._L.gvh_set_context(self._app, chain_id.encode(), height, int(recheck), gas_limit)

    def set_account(self, addr20: bytes, number: int, sequence: int, pub_amino: bytes = b""):
        self._L.gvh_set_account(self._app, addr20, number, sequence, pub_amino or None, len(pub_amino))

    def get_account(self, addr20: bytes):
        num, seq, ln = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_size_t()
        buf = ctypes.create_string_buffer(512)
        if not self._L.gvh_get_account(self._app, addr20, ctypes.byref(num), ctypes.byref(seq), buf, ctypes.byref(ln)):
            return None
        return {"number": num.value, "sequence": seq.value, "pub": buf.raw[:ln.value]}

    def ante(self, tx: bytes, simulate: bool = False):
        r = Result()
        rc = self._L.gvh_ante(self._app, tx, len(tx), int(simulate), ctypes.byref(r))
        return rc, r.as_dict()

    def preverify(self, txs):
        arr, lens = _arrays(txs)
        n = ctypes.c_size_t()
        rc = self._L.gvh_preverify(self._app, len(txs), arr, lens, ctypes.byref(n))
        return rc, n.value

    def deliver_block(self, txs):
        """(rc, [result dict per tx])"""
        arr, lens = _arrays(txs)
        res = (Result * max(1, len(txs)))()
        rc = self._L.gvh_deliver_block(self._app, len(txs), arr, lens, res)
        return rc, [res[i].as_dict() for i in range(len(txs))]

    def deliver_block_codes(self, txs):
        """Same, returning only (rc, numpy array of codes) -- cheap for large blocks."""
        import numpy as np
        arr, lens = _arrays(txs)
        codes = np.zeros(max(1, len(txs)), np.uint32)
        rc = self._L.gvh_deliver_block_codes(self._app, len(txs), arr, lens,
                                             codes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return rc, codes[:len(txs)]

    def deliver_block_blob(self, blob, offs, lens):
        """A block held in one contiguous buffer (numpy u8 blob, u64 offsets, u64
        lengths): no per-tx Python objects.  Returns (rc, codes u32 array)."""
        import numpy as np
        n = len(offs)
        ptrs = np.uint64(blob.ctypes.data) + offs.astype(np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        codes = np.zeros(max(1, n), np.uint32)
        rc = self._L.gvh_deliver_block_codes(self._app, n, ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)),
                                             lens.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)),
                                             codes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return rc, codes[:n]

    def deliver_blocks_blob(self, blob, offs, lens, block_ntx):
        """Consecutive blocks in one buffer (block b = the next block_ntx[b]
        txs of offs / lens), delivered through the pipelined replay
        (gvh_deliver_blocks): same codes and final state as deliver_block_blob
        per block.  Returns (rc, codes u32 array over every tx)."""
        import numpy as np
        n = len(offs)
        bn = np.ascontiguousarray(block_ntx, dtype=np.uint64)
        assert int(bn.sum()) == n
        ptrs = np.uint64(blob.ctypes.data) + np.asarray(offs).astype(np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        codes = np.zeros(max(1, n), np.uint32)
        rc = self._L.gvh_deliver_blocks(self._app, len(bn), bn.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)),
                                        ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)),
                                        lens.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)),
                                        codes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return rc, codes[:n]

    def deliver_blocks(self, blocks):
        """blocks: list of lists of tx bytes.  Returns (rc, [codes per block])."""
        import numpy as np
        flat = [tx for blk in blocks for tx in blk]
        lens = np.array([len(x) for x in flat], np.uint64)
        offs = np.zeros(len(flat), np.uint64)
        if len(flat):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(flat) or b"\0", np.uint8).copy()
        rc, codes = self.deliver_blocks_blob(blob, offs, lens, [len(b) for b in blocks])
        out, k = [], 0
        for b in blocks:
            out.append(codes[k:k + len(b)])
            k += len(b)
        return rc, out

    def deliver_gentxs(self, txs):
        arr, lens = _arrays(txs)
        res = (Result * max(1, len(txs)))()
        first = ctypes.c_size_t()
        rc = self._L.gvh_deliver_gentxs(self._app, len(txs), arr, lens, res, ctypes.byref(first))
        return rc, [res[i].as_dict() for i in range(len(txs))], first.value

    def checktx(self, tx: bytes):
        r = Result()
        rc = self._L.gvh_checktx(self._app, tx, len(tx), ctypes.byref(r))
        return rc, r.as_dict()

    def set_window(self, max_txs: int, max_wait_us: int):
        self._L.gvh_set_window(self._app, max_txs, max_wait_us)

    def set_cache_capacity(self, entries: int):
        self._L.gvh_set_cache_capacity(self._app, entries)

    def verify_commits(self, commits):
        """gvh_verify_commits over a list of dicts: vals = [(pub32, addr20, power)],
        sigs = [(flag, addr20, sig_bytes, sign_bytes)], trusting (bool),
        trust = (num, den), basic_ok (bool), keys_trusted (bool, default: trusting -- the
        trusted set of VerifyCommitTrusting; an adjacent VerifyCommit's set passes True).
        Returns [(code name, idx, idx2, got, needed)]."""
        import numpy as np
        keep = []
        arr = (Commit * max(1, len(commits)))()
        for c, d in enumerate(commits):
            vals, sigs = d["vals"], d["sigs"]
            vp32 = np.frombuffer(b"".join(v[0] for v in vals) or b"\0", np.uint8).copy()
            va20 = np.frombuffer(b"".join(v[1] for v in vals) or b"\0", np.uint8).copy()
            vpow = np.array([v[2] for v in vals] or [0], np.int64)
            flags = np.array([x[0] for x in sigs] or [0], np.uint8)
            sa20 = np.frombuffer(b"".join(x[1] for x in sigs) or b"\0", np.uint8).copy()
            s64 = np.zeros((max(1, len(sigs)), 64), np.uint8)
            slen = np.zeros(max(1, len(sigs)), np.uint32)
            for i, x in enumerate(sigs):
                b = x[2][:64]
                s64[i, :len(b)] = np.frombuffer(b, np.uint8) if b else 0
                slen[i] = len(x[2])
            msgs = [x[3] for x in sigs]
            blob = np.frombuffer(b"".join(msgs) or b"\0", np.uint8).copy()
            off = np.zeros(max(1, len(msgs)), np.uint64)
            ln = np.array([len(m) for m in msgs] or [0], np.uint32)
            if len(msgs) > 1:
                off[1:len(msgs)] = np.cumsum(ln[:len(msgs) - 1], dtype=np.uint64)
            keep += [vp32, va20, vpow, flags, sa20, s64, slen, blob, off, ln]
            num, den = d.get("trust", (1, 3))
            arr[c] = Commit(1 if d.get("trusting") else 0, num, den, 1 if d.get("basic_ok", True) else 0, len(vals),
                            vp32.ctypes.data, va20.ctypes.data, vpow.ctypes.data, len(sigs), flags.ctypes.data,
                            sa20.ctypes.data, s64.ctypes.data, slen.ctypes.data, blob.ctypes.data, off.ctypes.data,
                            ln.ctypes.data, 1 if d.get("keys_trusted", d.get("trusting")) else 0)
        res = (CommitResult * max(1, len(commits)))()
        rc = self._L.gvh_verify_commits(self._app, len(commits), arr, res)
        if rc != 0:
            raise RuntimeError(f"gvh_verify_commits rc {rc}")
        return [(COMMIT_CODES[r.code], r.idx, r.idx2, r.got, r.needed) for r in res[:len(commits)]]

    def stats(self):
        st = Stats()
        self._L.gvh_get_stats(self._app, ctypes.byref(st))
        return {k: getattr(st, k) for k, _ in Stats._fields_}

    def consume_sig_gas(self, sig: bytes, pub_amino: bytes | None, gas_limit: int = 0):
        r = Result()
        self._L.gvh_consume_sig_gas(self._app, sig, len(sig), pub_amino, len(pub_amino or b""), gas_limit,
                                    ctypes.byref(r))
        return r.as_dict()

    def set_threads(self, n: int):
        self._L.gvh_set_threads(self._app, n)

    def set_keyed(self, keyed: bool, load_min: int = 4096):
        """secp256k1 leaves through the GPU context's key arena (default; keys loaded by
        batches of >= load_min leaves) or as pub33 batches."""
        self._L.gvh_set_keyed(self._app, 1 if keyed else 0, load_min)

    def set_gpu_hash(self, on: bool):
        """delivered blocks with an empty verdict cache: secp256k1 sign bytes hashed
        in the GPU batch or on the host (default: measured faster)"""
        self._L.gvh_set_gpu_hash(self._app, 1 if on else 0)

    def gpu_hash(self) -> bool:
        return bool(self._L.gvh_get_gpu_hash(self._app))

    def keyed_policy(self):
        """(keyed, load_min, key_cap) in force"""
        k, lm, cap = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_size_t()
        self._L.gvh_get_keyed(self._app, ctypes.byref(k), ctypes.byref(lm), ctypes.byref(cap))
        return bool(k.value), lm.value, cap.value

    def cache_size(self) -> int:
        return self._L.gvh_cache_size(self._app)

    def cache_clear(self):
        self._L.gvh_cache_clear(self._app)
