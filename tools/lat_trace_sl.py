"""Phase breakdown of the sliced pub33 small-batch kernel (k_verify_lat_sl
built with GV_LAT_TRACE=1: `make ab NAME=trace DEFS=-DGV_LAT_TRACE=1`), 64
signatures per call.  Prints one JSON line of per-phase microseconds from the
block's start (median over blocks and repetitions)."""
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

MARKS = ["start", "key_decompressed", "tables_done", "scalars_done(wave1)", "after_barrier", "ladder_done",
         "combine_done", "end"]


def main():
    n = 64
    pub, sig, dig, exp = bench.make_digest_workload(4096, 0xC5, 256, 0.0, 16)
    ver = gvm.Verifier([0])
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 0     # 1: k_verify_lat_sl4 (mark 7: G sum done)
    ver.set_option("lat_rows_max", 1 << 30 if rows else 0)
    L = gvm._lib
    L.gv_debug_lat_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    acc = []
    for r in range(40):
        o = r * n
        got = ver.verify_batch_digests(pub[o:o + n], sig[o:o + n], dig[o:o + n])
        assert np.array_equal(got, exp[o:o + n])
        tr = np.zeros((n, 8), np.uint64)
        assert L.gv_debug_lat_trace(tr.ctypes.data, n) == 0
        t = tr.astype(np.int64)
        acc.append((t - t[:, :1]) * 0.01)            # 100 MHz ticks -> us from the block's start
    a = np.concatenate(acc[5:])
    med = np.median(a, 0)
    ver.close()
    marks = MARKS[:7] + (["g_sum_done(wave1)"] if rows else MARKS[7:])
    print(json.dumps({"kernel": "k_verify_lat_sl4" if rows else "k_verify_lat_sl",
                      **{k: round(float(v), 2) for k, v in zip(marks, med)}}))


if __name__ == "__main__":
    main()
