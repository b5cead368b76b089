"""PreVerifyTxs host-stage timing (no GPU work: HostApp without a verifier
stops after the cache lookup) for 10k MsgSend txs at several thread counts.
Run with GVH_PROFILE=1 for the per-stage lines on stderr."""
import struct
import sys
import time
import os
import ctypes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import gvhost  # noqa: E402
import txkit as T  # noqa: E402

ntx = 10000
keys = []
for i in range(ntx + 1):
    priv = T.privkey_from_secret(b"gv-c1-" + struct.pack("<Q", i))
    amino = T.amino_secp(T.secp_pubkey(priv))
    keys.append((priv, amino, T.address(amino)))
fee = T.fee_json([(0, "stake")], 1000000)
txs = []
for i in range(ntx):
    priv, amino, addr = keys[i]
    msg = T.msg_send_json(addr, keys[i + 1][2], [(10, "foocoin")])
    txs.append(T.flat_tx([msg], fee, "", [addr], [(amino, b"\x01" * 64)]))
app = gvhost.HostApp(None, chain_id="gv-bench", height=1)
for i in range(ntx):
    app.set_account(keys[i][2], i, 0)
arr = (ctypes.c_char_p * len(txs))(*txs)
lens = (ctypes.c_size_t * len(txs))(*[len(t) for t in txs])
n = ctypes.c_size_t()
for th in (1, 4, 8, 16, 1, 16):
    app.set_threads(th)
    t = time.perf_counter()
    app._L.gvh_preverify(app._app, len(txs), arr, lens, ctypes.byref(n))
    print(th, "threads", round((time.perf_counter() - t) * 1e3, 2), "ms", flush=True)
