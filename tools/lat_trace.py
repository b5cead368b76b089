"""Phase breakdown of the fused small-batch kernel (gv_lat.hip built with
GV_LAT_TRACE=1: `make ab NAME=trace DEFS=-DGV_LAT_TRACE=1`), 64-signature
batches, pub33 and keyed.  Prints one JSON line of per-phase microseconds
(median over blocks and repetitions)."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GV_LIB", os.path.join(REPO, "cosmos-sdk-rootchain_amd", "lib", "libgpuverify_trace.so"))
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402

PHASES = ["wave0_prep", "wave1_scalars", "barrier_after_both", "ladder", "combine", "final_check",
          "total_in_kernel", "wave0_sqrt"]


def main():
    n = 64
    pub, sig, dig, exp = bench.make_digest_workload(4096, 0xC5, 256, 0.0, 16)
    ver = gvm.Verifier([0])
    L = gvm._lib
    L.gv_debug_lat_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    slots = ver.keys_load(pub[:256])[np.arange(len(pub)) % 256]
    out = {}
    for mode in ("pub33", "keyed"):
        rows = []
        for r in range(30):
            o = r * n
            if mode == "pub33":
                got = ver.verify_batch_digests(pub[o:o + n], sig[o:o + n], dig[o:o + n])
            else:
                got = ver.verify_batch_digests_keyed(slots[o:o + n], sig[o:o + n], dig[o:o + n])
            assert np.array_equal(got, exp[o:o + n])
            tr = np.zeros((n // 16, 8), np.uint64)
            assert L.gv_debug_lat_trace(tr.ctypes.data, n // 16) == 0
            t = tr.astype(np.int64)
            rows.append(np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 0], t[:, 3] - t[:, 0], t[:, 4] - t[:, 3],
                                  t[:, 5] - t[:, 4], t[:, 6] - t[:, 5], t[:, 6] - t[:, 0],
                                  (t[:, 7] - t[:, 0]) if mode == "pub33" else 0 * t[:, 0]], 1))
        a = np.concatenate(rows[5:]) * 0.01          # 100 MHz ticks -> us
        med = np.median(a, 0)
        out[mode] = {k: round(float(v), 2) for k, v in zip(PHASES, med)}
    ver.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
