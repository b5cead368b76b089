"""gpuverify.py -- ctypes binding of libgpuverify.so (include/gpuverify.h).

Host-side mirror of the reference's verification interface for tests and the
benchmark (the reference's own host language, Go, has no toolchain in this
image; INTEGRATION.md carries the cgo binding).  Names follow the reference:

  PubKeySecp256k1(pub33).verify_bytes(msg, sig)   tendermint VerifyBytes
                                                  (x/auth/ante/sigverify.go:210)
  Verifier.verify_batch_msgs / verify_batch_digests   batched VerifyBytes
                                                  (crypto/gpuverify in INTEGRATION.md)

This module never falls back to a CPU implementation: if libgpuverify.so is
missing or no HIP device is present it raises GpuVerifyError.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GV_LIB overrides the library path (A/B runs of alternative builds); the default
# is the in-tree build.
# defaults of the "lat_max" / "lat_sl_max" options (gv_runtime.cpp): the small-batch / pipeline
# crossover and the sliced / four-lanes-per-signature small-batch crossover
LAT_MAX_DEFAULT = 8192
LAT_SL_MAX_DEFAULT = 2048
LAT_ROWS_MAX_DEFAULT = 512        # pub33 batches up to this many: k_verify_lat_sl4 ("lat_rows_max")
# keyed batches: their own defaults (setting "lat_max" / "lat_sl_max" sets the keyed ones too)
LAT_MAX_KEYED_DEFAULT = 14336
LAT_SL_MAX_KEYED_DEFAULT = 1536
LIB_PATH = os.environ.get("GV_LIB") or os.path.join(HERE, "lib", "libgpuverify.so")

GV_OK, GV_EINVAL, GV_ENODEV, GV_EHIP, GV_ENOMEM, GV_EFAULT = 0, -1, -2, -3, -4, -5

# every symbol include/gpuverify.h declares
EXPORTED_SYMBOLS = (
    "gv_open", "gv_close", "gv_num_devices", "gv_verify_msgs", "gv_verify_digests",
    "gv_verify_digests_bits", "gv_verify_msgs_bits", "gv_dev_verify_digests", "gv_dev_verify_msgs",
    "gv_set_option", "gv_get_option", "gv_last_stage_ms", "gv_strerror", "gv_debug_op", "gv_dev_alloc", "gv_dev_free",
    "gv_dev_copy", "gv_dev_sync", "gv_stage_stats", "gv_keys_load", "gv_keys_reset", "gv_keys_count", "gv_keys_generation",
    "gv_verify_digests_keyed", "gv_verify_msgs_keyed", "gv_dev_verify_digests_keyed", "gv_stage_stats4",
    "gv_keys_point", "gv_dev_stream_create", "gv_dev_stream_sync", "gv_dev_stream_destroy",
    "gv_verify_ed25519_msgs", "gv_dev_verify_ed25519_msgs", "gv_last_slices", "gv_group_stats", "gv_route_stats", "gv_host_alloc", "gv_host_free",
    "gv_ed_keys_load", "gv_ed_keys_reset", "gv_ed_keys_count", "gv_ed_keys_generation", "gv_verify_ed25519_msgs_keyed",
    "gv_submit_digests", "gv_submit_digests_keyed", "gv_submit_msgs", "gv_submit_msgs_keyed", "gv_wait",
)


class GpuVerifyError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _strerror(code) if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def load(path: str = LIB_PATH):
    """Load libgpuverify.so and declare argtypes.  Does not touch the GPU."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GpuVerifyError(GV_ENODEV, f"{path} not built (run make -C {HERE})")
    L = ctypes.CDLL(path)
    vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.gv_open.argtypes = [ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.gv_open.restype = i32
    L.gv_close.argtypes = [vp]
    L.gv_close.restype = None
    L.gv_num_devices.argtypes = [vp]
    L.gv_num_devices.restype = i32
    L.gv_verify_msgs.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp]
    L.gv_verify_msgs.restype = i32
    L.gv_verify_digests.argtypes = [vp, sz, vp, vp, vp, vp]
    L.gv_verify_digests.restype = i32
    L.gv_verify_digests_bits.argtypes = [vp, sz, vp, vp, vp, vp]
    L.gv_verify_digests_bits.restype = i32
    L.gv_verify_msgs_bits.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp]
    L.gv_verify_msgs_bits.restype = i32
    L.gv_dev_verify_digests.argtypes = [vp, i32, sz, vp, vp, vp, vp, vp]
    L.gv_dev_verify_digests.restype = i32
    L.gv_dev_verify_msgs.argtypes = [vp, i32, sz, vp, vp, vp, vp, vp, vp, vp]
    L.gv_dev_verify_msgs.restype = i32
    L.gv_verify_ed25519_msgs.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp]
    L.gv_verify_ed25519_msgs.restype = i32
    L.gv_dev_verify_ed25519_msgs.argtypes = [vp, i32, sz, vp, vp, vp, vp, vp, vp, vp]
    L.gv_dev_verify_ed25519_msgs.restype = i32
    L.gv_ed_keys_load.argtypes = [vp, sz, vp, vp]
    L.gv_ed_keys_load.restype = i32
    L.gv_ed_keys_reset.argtypes = [vp]
    L.gv_ed_keys_reset.restype = i32
    L.gv_ed_keys_count.argtypes = [vp]
    L.gv_ed_keys_count.restype = sz
    L.gv_ed_keys_generation.argtypes = [vp]
    L.gv_ed_keys_generation.restype = ctypes.c_uint64
    L.gv_verify_ed25519_msgs_keyed.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp]
    L.gv_verify_ed25519_msgs_keyed.restype = i32
    L.gv_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_longlong]
    L.gv_set_option.restype = i32
    L.gv_get_option.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)]
    L.gv_get_option.restype = i32
    L.gv_last_stage_ms.argtypes = [vp, i32] + [ctypes.POINTER(ctypes.c_float)] * 3
    L.gv_last_stage_ms.restype = i32
    L.gv_strerror.argtypes = [i32]
    L.gv_strerror.restype = ctypes.c_char_p
    L.gv_debug_op.argtypes = [vp, i32, i32, sz, vp, vp]
    L.gv_debug_op.restype = i32
    L.gv_dev_alloc.argtypes = [vp, i32, sz, ctypes.POINTER(vp)]
    L.gv_dev_alloc.restype = i32
    L.gv_dev_free.argtypes = [vp, i32, vp]
    L.gv_dev_free.restype = i32
    L.gv_dev_copy.argtypes = [vp, i32, vp, vp, sz, i32]
    L.gv_dev_copy.restype = i32
    L.gv_dev_sync.argtypes = [vp, i32]
    L.gv_dev_sync.restype = i32
    L.gv_dev_stream_create.argtypes = [vp, i32, ctypes.POINTER(vp)]
    L.gv_dev_stream_create.restype = i32
    L.gv_dev_stream_sync.argtypes = [vp, i32, vp]
    L.gv_dev_stream_sync.restype = i32
    L.gv_dev_stream_destroy.argtypes = [vp, i32, vp]
    L.gv_dev_stream_destroy.restype = i32
    L.gv_stage_stats.argtypes = [vp, i32, ctypes.POINTER(i32)] + [ctypes.POINTER(ctypes.c_double)] * 3
    L.gv_stage_stats.restype = i32
    L.gv_stage_stats4.argtypes = [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double)]
    L.gv_stage_stats4.restype = i32
    L.gv_last_slices.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_size_t), i32]
    L.gv_last_slices.restype = i32
    L.gv_group_stats.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.gv_group_stats.restype = i32
    L.gv_route_stats.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_uint64)]
    L.gv_route_stats.restype = i32
    L.gv_host_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    L.gv_host_alloc.restype = i32
    L.gv_host_free.argtypes = [vp, vp]
    L.gv_host_free.restype = i32
    L.gv_keys_load.argtypes = [vp, sz, vp, vp]
    L.gv_keys_load.restype = i32
    L.gv_keys_reset.argtypes = [vp]
    L.gv_keys_reset.restype = i32
    L.gv_keys_count.argtypes = [vp]
    L.gv_keys_count.restype = sz
    L.gv_keys_generation.argtypes = [vp]
    L.gv_keys_generation.restype = ctypes.c_uint64
    L.gv_keys_point.argtypes = [vp, sz, vp, vp, vp]
    L.gv_keys_point.restype = i32
    L.gv_verify_digests_keyed.argtypes = [vp, sz, vp, vp, vp, vp]
    L.gv_verify_digests_keyed.restype = i32
    L.gv_verify_msgs_keyed.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp]
    L.gv_verify_msgs_keyed.restype = i32
    L.gv_dev_verify_digests_keyed.argtypes = [vp, i32, sz, vp, vp, vp, vp, vp]
    L.gv_dev_verify_digests_keyed.restype = i32
    u64p = ctypes.POINTER(ctypes.c_uint64)
    for name, nargs in (("gv_submit_digests", 4), ("gv_submit_digests_keyed", 4), ("gv_submit_msgs", 6),
                        ("gv_submit_msgs_keyed", 6)):
        getattr(L, name).argtypes = [vp, sz] + [vp] * nargs + [u64p]
        getattr(L, name).restype = i32
    L.gv_wait.argtypes = [vp, ctypes.c_uint64]
    L.gv_wait.restype = i32
    _lib = L
    return L


def _strerror(code: int) -> str:
    return _lib.gv_strerror(code).decode()


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def _check(rc: int, what: str):
    if rc != GV_OK:
        raise GpuVerifyError(rc, what)


def pack_msgs(msgs):
    """list[bytes] -> (blob u8, off u64, len u32)"""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=len(msgs))
    off = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs) > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
    return blob, off, lens


class Verifier:
    """Batched VerifyBytes on one or more MI355X devices (gv_ctx)."""

    def __init__(self, devices=None):
        L = load()
        ctx = ctypes.c_void_p()
        if devices:
            ids = (ctypes.c_int * len(devices))(*devices)
            rc = L.gv_open(ids, len(devices), ctypes.byref(ctx))
        else:
            rc = L.gv_open(None, 0, ctypes.byref(ctx))
        _check(rc, "gv_open")
        self._ctx = ctx
        self._L = L
        # submitted batches not yet waited for: ticket -> (input arrays, verdicts).
        # The library reads the inputs and writes the verdicts until gv_wait, so
        # they live here, not only in the Pending the caller may drop.
        self._inflight = {}

    def close(self):
        if self._ctx:
            for t in list(self._inflight):        # the lanes use these buffers until each batch is done
                self._release(t)
            self._L.gv_close(self._ctx)
            self._ctx = None

    def _release(self, ticket) -> int:
        """gv_wait on a ticket still in flight (a dropped Pending, close()); 0 if already waited."""
        if ticket not in self._inflight or not self._ctx:
            return 0
        rc = self._L.gv_wait(self._ctx, ticket)
        self._inflight.pop(ticket, None)
        return rc

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_devices(self) -> int:
        return self._L.gv_num_devices(self._ctx)

    def reset_schedule(self):
        """The small-batch schedule options back to their defaults."""
        self.set_option("lat_max", LAT_MAX_DEFAULT)
        self.set_option("lat_sl_max", LAT_SL_MAX_DEFAULT)
        self.set_option("lat_max_keyed", LAT_MAX_KEYED_DEFAULT)
        self.set_option("lat_sl_max_keyed", LAT_SL_MAX_KEYED_DEFAULT)
        self.set_option("lat_rows_max", LAT_ROWS_MAX_DEFAULT)

    def set_option(self, key: str, val: int):
        _check(self._L.gv_set_option(self._ctx, key.encode(), int(val)), f"gv_set_option({key})")

    def get_option(self, key: str) -> int:
        v = ctypes.c_longlong(0)
        _check(self._L.gv_get_option(self._ctx, key.encode(), ctypes.byref(v)), f"gv_get_option({key})")
        return int(v.value)

    def verify_batch_digests(self, pub33: np.ndarray, sig64: np.ndarray, dig32: np.ndarray) -> np.ndarray:
        pub33, sig64, dig32 = (np.ascontiguousarray(a, dtype=np.uint8) for a in (pub33, sig64, dig32))
        n = pub33.shape[0]
        assert pub33.shape == (n, 33) and sig64.shape == (n, 64) and dig32.shape == (n, 32)
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_digests(self._ctx, n, _ptr(pub33), _ptr(sig64), _ptr(dig32), _ptr(out)),
                   "gv_verify_digests")
        return out

    def verify_batch_digests_bits(self, pub33, sig64, dig32) -> np.ndarray:
        n = pub33.shape[0]
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        if n:
            _check(self._L.gv_verify_digests_bits(self._ctx, n, _ptr(pub33), _ptr(sig64), _ptr(dig32),
                                                  _ptr(out)), "gv_verify_digests_bits")
        return out

    def verify_batch_msgs(self, pub33: np.ndarray, sig64: np.ndarray, msgs) -> np.ndarray:
        """msgs: list[bytes] or a (blob, off, len) triple."""
        pub33, sig64 = (np.ascontiguousarray(a, dtype=np.uint8) for a in (pub33, sig64))
        blob, off, ln = pack_msgs(msgs) if isinstance(msgs, (list, tuple)) and (
            len(msgs) == 0 or isinstance(msgs[0], (bytes, bytearray))) else msgs
        n = pub33.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_msgs(self._ctx, n, _ptr(pub33), _ptr(sig64), _ptr(blob), _ptr(off),
                                          _ptr(ln), _ptr(out)), "gv_verify_msgs")
        return out

    # ---- asynchronous host batches (gv_submit_* / gv_wait)
    class Pending:
        """A submitted batch: its ticket and verdict array.  The Verifier keeps
        the input arrays (and the verdicts) alive until the batch is waited for;
        a Pending dropped without wait() is waited for when it is collected, so
        the library never touches freed memory."""
        def __init__(self, ticket, out):
            self.ticket, self.out = ticket, out

    def _submit(self, fn, name, n, args, keep):
        out = np.zeros(n, dtype=np.uint8)
        t = ctypes.c_uint64(0)
        _check(fn(self._ctx, n, *[_ptr(a) for a in args], _ptr(out), ctypes.byref(t)), name)
        self._inflight[t.value] = (keep, out)
        p = Verifier.Pending(t.value, out)
        weakref.finalize(p, self._release, t.value)
        return p

    def submit_digests(self, pub33, sig64, dig32) -> "Verifier.Pending":
        a = [np.ascontiguousarray(x, dtype=np.uint8) for x in (pub33, sig64, dig32)]
        return self._submit(self._L.gv_submit_digests, "gv_submit_digests", a[0].shape[0], a, a)

    def submit_digests_keyed(self, slots, sig64, dig32) -> "Verifier.Pending":
        a = [np.ascontiguousarray(slots, dtype=np.uint32)] + [np.ascontiguousarray(x, dtype=np.uint8)
                                                             for x in (sig64, dig32)]
        return self._submit(self._L.gv_submit_digests_keyed, "gv_submit_digests_keyed", a[0].shape[0], a, a)

    def submit_msgs(self, pub33, sig64, msgs, slots=None) -> "Verifier.Pending":
        blob, off, ln = pack_msgs(msgs) if isinstance(msgs, (list, tuple)) and (
            len(msgs) == 0 or isinstance(msgs[0], (bytes, bytearray))) else msgs
        sig64 = np.ascontiguousarray(sig64, dtype=np.uint8)
        if slots is not None:
            k = np.ascontiguousarray(slots, dtype=np.uint32)
            a = [k, sig64, blob, off, ln]
            return self._submit(self._L.gv_submit_msgs_keyed, "gv_submit_msgs_keyed", k.shape[0], a, a)
        p = np.ascontiguousarray(pub33, dtype=np.uint8)
        a = [p, sig64, blob, off, ln]
        return self._submit(self._L.gv_submit_msgs, "gv_submit_msgs", p.shape[0], a, a)

    def wait(self, pending: "Verifier.Pending") -> np.ndarray:
        if pending.ticket not in self._inflight:
            raise GpuVerifyError(GV_EINVAL, "gv_wait: ticket already waited for")
        rc = self._L.gv_wait(self._ctx, pending.ticket)
        self._inflight.pop(pending.ticket, None)
        _check(rc, "gv_wait")
        return pending.out

    # ---- account pubkey cache (gv_keys_*)
    def keys_load(self, pub33: np.ndarray) -> np.ndarray:
        """Parse and keep n keys resident; returns their slots (u32)."""
        pub33 = np.ascontiguousarray(pub33, dtype=np.uint8)
        n = pub33.shape[0]
        assert pub33.shape == (n, 33)
        slots = np.zeros(n, dtype=np.uint32)
        if n:
            _check(self._L.gv_keys_load(self._ctx, n, _ptr(pub33), _ptr(slots)), "gv_keys_load")
        return slots

    def keys_point(self, slots: np.ndarray):
        """Affine points (n x 64 bytes x||y) and ParsePubKey verdicts the key arena holds for `slots`."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        n = slots.shape[0]
        xy = np.zeros((n, 64), dtype=np.uint8)
        ok = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_keys_point(self._ctx, n, _ptr(slots), _ptr(xy), _ptr(ok)), "gv_keys_point")
        return xy, ok

    def keys_reset(self):
        _check(self._L.gv_keys_reset(self._ctx), "gv_keys_reset")

    @property
    def keys_count(self) -> int:
        return self._L.gv_keys_count(self._ctx)

    def verify_batch_digests_keyed(self, slots: np.ndarray, sig64: np.ndarray, dig32: np.ndarray) -> np.ndarray:
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        sig64, dig32 = (np.ascontiguousarray(a, dtype=np.uint8) for a in (sig64, dig32))
        n = slots.shape[0]
        assert sig64.shape == (n, 64) and dig32.shape == (n, 32)
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_digests_keyed(self._ctx, n, _ptr(slots), _ptr(sig64), _ptr(dig32), _ptr(out)),
                   "gv_verify_digests_keyed")
        return out

    def verify_batch_msgs_keyed(self, slots: np.ndarray, sig64: np.ndarray, msgs) -> np.ndarray:
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        sig64 = np.ascontiguousarray(sig64, dtype=np.uint8)
        blob, off, ln = pack_msgs(msgs) if isinstance(msgs, (list, tuple)) and (
            len(msgs) == 0 or isinstance(msgs[0], (bytes, bytearray))) else msgs
        n = slots.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_msgs_keyed(self._ctx, n, _ptr(slots), _ptr(sig64), _ptr(blob), _ptr(off),
                                                _ptr(ln), _ptr(out)), "gv_verify_msgs_keyed")
        return out

    def dev_verify_digests_keyed(self, slot: int, n: int, d_slots, d_sig, d_dig, d_bits, stream=None):
        _check(self._L.gv_dev_verify_digests_keyed(self._ctx, slot, n, ctypes.c_void_p(d_slots),
                                                   ctypes.c_void_p(d_sig), ctypes.c_void_p(d_dig),
                                                   ctypes.c_void_p(d_bits), ctypes.c_void_p(stream or 0)),
               "gv_dev_verify_digests_keyed")

    def dev_verify_digests(self, slot: int, n: int, d_pub, d_sig, d_dig, d_bits, stream=None):
        """Device-resident path: d_* are device addresses (ints); stream a hipStream_t int."""
        _check(self._L.gv_dev_verify_digests(self._ctx, slot, n, ctypes.c_void_p(d_pub), ctypes.c_void_p(d_sig),
                                             ctypes.c_void_p(d_dig), ctypes.c_void_p(d_bits),
                                             ctypes.c_void_p(stream or 0)), "gv_dev_verify_digests")

    def dev_verify_msgs(self, slot: int, n: int, d_pub, d_sig, d_blob, d_off, d_len, d_bits, stream=None):
        _check(self._L.gv_dev_verify_msgs(self._ctx, slot, n, ctypes.c_void_p(d_pub), ctypes.c_void_p(d_sig),
                                          ctypes.c_void_p(d_blob), ctypes.c_void_p(d_off), ctypes.c_void_p(d_len),
                                          ctypes.c_void_p(d_bits), ctypes.c_void_p(stream or 0)),
               "gv_dev_verify_msgs")

    # ---- ed25519
    def verify_batch_ed25519(self, pub32: np.ndarray, sig64: np.ndarray, msgs) -> np.ndarray:
        """out[i] = PubKeyEd25519(pub32[i]).VerifyBytes(msg_i, sig64[i]); msgs: list[bytes] or
        a (blob, off, len) triple."""
        pub32, sig64 = (np.ascontiguousarray(a, dtype=np.uint8) for a in (pub32, sig64))
        blob, off, ln = pack_msgs(msgs) if isinstance(msgs, (list, tuple)) and (
            len(msgs) == 0 or isinstance(msgs[0], (bytes, bytearray))) else msgs
        n = pub32.shape[0]
        assert pub32.shape == (n, 32) and sig64.shape == (n, 64) and len(off) == n and len(ln) == n
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_ed25519_msgs(self._ctx, n, _ptr(pub32), _ptr(sig64), _ptr(blob),
                                                  _ptr(np.ascontiguousarray(off, dtype=np.uint64)),
                                                  _ptr(np.ascontiguousarray(ln, dtype=np.uint32)), _ptr(out)),
                   "gv_verify_ed25519_msgs")
        return out

    def ed_keys_load(self, pub32: np.ndarray) -> np.ndarray:
        """FromBytes + the comb table of -A, kept resident per key; returns the slots (u32)."""
        pub32 = np.ascontiguousarray(pub32, dtype=np.uint8)
        n = pub32.shape[0]
        assert pub32.shape == (n, 32)
        slots = np.zeros(n, dtype=np.uint32)
        if n:
            _check(self._L.gv_ed_keys_load(self._ctx, n, _ptr(pub32), _ptr(slots)), "gv_ed_keys_load")
        return slots

    def ed_keys_reset(self):
        _check(self._L.gv_ed_keys_reset(self._ctx), "gv_ed_keys_reset")

    @property
    def ed_keys_count(self) -> int:
        return self._L.gv_ed_keys_count(self._ctx)

    @property
    def ed_keys_generation(self) -> int:
        return self._L.gv_ed_keys_generation(self._ctx)

    def verify_batch_ed25519_keyed(self, slots: np.ndarray, sig64: np.ndarray, msgs) -> np.ndarray:
        """verify_batch_ed25519 with the key of each item given by its ed25519 key-arena slot."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        sig64 = np.ascontiguousarray(sig64, dtype=np.uint8)
        blob, off, ln = pack_msgs(msgs) if isinstance(msgs, (list, tuple)) and (
            len(msgs) == 0 or isinstance(msgs[0], (bytes, bytearray))) else msgs
        n = slots.shape[0]
        assert sig64.shape == (n, 64) and len(off) == n and len(ln) == n
        out = np.zeros(n, dtype=np.uint8)
        if n:
            _check(self._L.gv_verify_ed25519_msgs_keyed(self._ctx, n, _ptr(slots), _ptr(sig64), _ptr(blob),
                                                        _ptr(np.ascontiguousarray(off, dtype=np.uint64)),
                                                        _ptr(np.ascontiguousarray(ln, dtype=np.uint32)), _ptr(out)),
                   "gv_verify_ed25519_msgs_keyed")
        return out

    def dev_verify_ed25519(self, slot: int, n: int, d_pub, d_sig, d_blob, d_off, d_len, d_bits, stream=None):
        _check(self._L.gv_dev_verify_ed25519_msgs(self._ctx, slot, n, ctypes.c_void_p(d_pub), ctypes.c_void_p(d_sig),
                                                  ctypes.c_void_p(d_blob), ctypes.c_void_p(d_off),
                                                  ctypes.c_void_p(d_len), ctypes.c_void_p(d_bits),
                                                  ctypes.c_void_p(stream or 0)), "gv_dev_verify_ed25519_msgs")

    def last_stage_ms(self, slot: int = 0):
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _check(self._L.gv_last_stage_ms(self._ctx, slot, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
               "gv_last_stage_ms")
        return a.value, b.value, c.value

    # ---- device memory helpers (no torch/HIP runtime needed on the caller side)
    def dev_alloc(self, nbytes: int, slot: int = 0) -> int:
        p = ctypes.c_void_p()
        _check(self._L.gv_dev_alloc(self._ctx, slot, nbytes, ctypes.byref(p)), "gv_dev_alloc")
        return p.value

    def dev_free(self, ptr: int, slot: int = 0):
        _check(self._L.gv_dev_free(self._ctx, slot, ctypes.c_void_p(ptr)), "gv_dev_free")

    def dev_upload(self, ptr: int, arr: np.ndarray, slot: int = 0):
        arr = np.ascontiguousarray(arr)
        _check(self._L.gv_dev_copy(self._ctx, slot, ctypes.c_void_p(ptr), _ptr(arr), arr.nbytes, 1), "gv_dev_copy")

    def dev_download(self, arr: np.ndarray, ptr: int, slot: int = 0):
        assert arr.flags["C_CONTIGUOUS"]
        _check(self._L.gv_dev_copy(self._ctx, slot, _ptr(arr), ctypes.c_void_p(ptr), arr.nbytes, 2), "gv_dev_copy")

    def dev_sync(self, slot: int = 0):
        _check(self._L.gv_dev_sync(self._ctx, slot), "gv_dev_sync")

    def stream_create(self, slot: int = 0) -> int:
        p = ctypes.c_void_p()
        _check(self._L.gv_dev_stream_create(self._ctx, slot, ctypes.byref(p)), "gv_dev_stream_create")
        return p.value

    def stream_sync(self, stream: int, slot: int = 0):
        _check(self._L.gv_dev_stream_sync(self._ctx, slot, ctypes.c_void_p(stream)), "gv_dev_stream_sync")

    def stream_destroy(self, stream: int, slot: int = 0):
        _check(self._L.gv_dev_stream_destroy(self._ctx, slot, ctypes.c_void_p(stream)), "gv_dev_stream_destroy")

    def stage_stats(self, slot: int = 0):
        c = ctypes.c_int()
        a, b, d = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _check(self._L.gv_stage_stats(self._ctx, slot, ctypes.byref(c), ctypes.byref(a), ctypes.byref(b),
                                      ctypes.byref(d)), "gv_stage_stats")
        return c.value, a.value, b.value, d.value

    def stage_stats4(self, slot: int = 0):
        """(count, [unpack/sha, scalar_inv, prep, ecmult] ms averaged over the launches since the last call)."""
        c = ctypes.c_int()
        ms = (ctypes.c_double * 4)()
        _check(self._L.gv_stage_stats4(self._ctx, slot, ctypes.byref(c), ms), "gv_stage_stats4")
        return c.value, list(ms)

    def host_array(self, shape, dtype=np.uint8):
        """A numpy array in pinned host memory (gv_host_alloc): host-buffer digest
        calls on such arrays skip the staging copy.  Freed with host_free(arr)."""
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = ctypes.c_void_p()
        _check(self._L.gv_host_alloc(self._ctx, max(1, nbytes), ctypes.byref(p)), "gv_host_alloc")
        buf = (ctypes.c_uint8 * max(1, nbytes)).from_address(p.value)
        arr = np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dtype).reshape(shape)
        self._pinned = getattr(self, "_pinned", {})
        self._pinned[arr.ctypes.data] = p.value
        return arr

    def host_free(self, arr):
        p = self._pinned.pop(arr.ctypes.data)
        _check(self._L.gv_host_free(self._ctx, p), "gv_host_free")

    def group_stats(self, slot: int = 0):
        """(batches that took the in-batch key grouping, distinct keys built) on device slot."""
        b, k = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.gv_group_stats(self._ctx, slot, ctypes.byref(b), ctypes.byref(k)), "gv_group_stats")
        return b.value, k.value

    KG_DEFAULT = 0         # gv_runtime.cpp gv_ctx::kg (the grouped route's default layout)
    ROUTES = ("pub33", "keyed125", "k4", "k6", "lat", "lat_keyed", "k4f", "item_f", "kn", "ed_lat", "kw", "kw2", "kg")

    def route_stats(self, slot: int = 0) -> dict:
        """Batches per secp256k1 schedule on device slot since open (gv_route_stats)."""
        out = (ctypes.c_uint64 * len(self.ROUTES))()
        _check(self._L.gv_route_stats(self._ctx, slot, out), "gv_route_stats")
        return dict(zip(self.ROUTES, (int(v) for v in out)))

    def last_slices(self):
        """[(ms, items)] per device slot: each device's slice of the last host-buffer call."""
        nd = self.num_devices
        ms = (ctypes.c_double * max(1, nd))()
        nn = (ctypes.c_size_t * max(1, nd))()
        m = self._L.gv_last_slices(self._ctx, ms, nn, nd)
        if m < 0:
            raise GpuVerifyError(m, "gv_last_slices")
        return [(ms[k], nn[k]) for k in range(m)]

    def debug_op(self, op: int, words: np.ndarray, slot: int = 0) -> np.ndarray:
        words = np.ascontiguousarray(words, dtype=np.uint32)
        n = words.shape[0]
        assert words.shape == (n, 16)
        out = np.zeros((n, 16), dtype=np.uint32)
        _check(self._L.gv_debug_op(self._ctx, slot, op, n, _ptr(words), _ptr(out)), "gv_debug_op")
        return out


class PubKeySecp256k1:
    """Mirror of tendermint crypto/secp256k1.PubKeySecp256k1 ([33]byte) whose
    VerifyBytes runs on the GPU (batch of one).  Same argument meaning and
    result: bool, never an exception for a cryptographic rejection."""

    _shared = None

    def __init__(self, pub33: bytes):
        assert len(pub33) == 33
        self.key = bytes(pub33)

    @classmethod
    def _verifier(cls):
        if cls._shared is None:
            cls._shared = Verifier()
        return cls._shared

    def verify_bytes(self, msg: bytes, sig: bytes) -> bool:
        if len(sig) != 64:          # VerifyBytes' first check, decided on the host
            return False
        pub = np.frombuffer(self.key, dtype=np.uint8).reshape(1, 33)
        s = np.frombuffer(bytes(sig), dtype=np.uint8).reshape(1, 64)
        return bool(self._verifier().verify_batch_msgs(pub, s, [bytes(msg)])[0])
