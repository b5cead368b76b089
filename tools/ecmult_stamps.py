"""Where does k_ecmult's time go at the C2 batch?  Runs the headline step
(gv_dev_verify_digests on a device-resident batch) with the diagnostic build
(lib/libgpuverify_stamp.so: `make -C cosmos-sdk-rootchain_amd ab NAME=stamp
DEFS=-DGV_STAMP=1`) and reads every k_ecmult wave's start / end shader clock,
100 MHz real time, SIMD / CU / XCD.  Reports, per batch size: the in-kernel
clock (d s_memtime / d s_memrealtime), the wave-duration distribution by
round, the launch-to-first-wave and last-wave tails, how busy the SIMDs are
over the kernel (wave-slots occupied / available), and the part of the
kernel spent after the last full round.
usage: ecmult_stamps.py [n1,n2,...] [out.json]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GV_LIB", os.path.join(REPO, "cosmos-sdk-rootchain_amd", "lib", "libgpuverify_stamp.so"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402


def analyse(st, nw):
    t0, t1, r0, r1, hw = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
    xcc = (hw >> 32) & 0xF
    hwid = hw & 0xFFFFFFFF
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 0xF
    se = (hwid >> 13) & 7
    clk_mhz = float(np.median((t1 - t0) / np.maximum(r1 - r0, 1)) * 100.0)
    # real time in microseconds from the first wave's start
    start = (r0 - r0.min()) / 100.0
    end = (r1 - r0.min()) / 100.0
    dur = end - start
    span = float(end.max())
    slot = xcc * 1000 + se * 100 + cu * 4 + simd          # a SIMD id
    nsimd = len(np.unique(slot))
    per_simd = np.bincount(np.unique(slot, return_inverse=True)[1])
    occ = float(dur.sum() / (span * nsimd))              # mean resident waves per SIMD over the kernel
    order = np.argsort(start)
    first_round = dur[order[: 3 * nsimd]]
    last_end = np.sort(end)
    # time at which the machine stops being full: the (3*nsimd)-th last end
    full_until = float(last_end[-3 * nsimd]) if nw > 3 * nsimd else 0.0
    return {"waves": int(nw), "simds_seen": int(nsimd), "xcds": int(len(np.unique(xcc))),
            "clock_mhz_median": round(clk_mhz, 1), "kernel_span_us": round(span, 1),
            "wave_us": {"p5": round(float(np.percentile(dur, 5)), 1), "p50": round(float(np.median(dur)), 1),
                        "p95": round(float(np.percentile(dur, 95)), 1), "max": round(float(dur.max()), 1)},
            "first_round_wave_us_p50": round(float(np.median(first_round)), 1),
            "waves_per_simd": {"min": int(per_simd.min()), "max": int(per_simd.max()),
                               "mean": round(float(per_simd.mean()), 2)},
            "mean_resident_waves_per_simd": round(occ, 3),
            "last_start_us": round(float(start.max()), 1),
            "tail_after_full_us": round(span - full_until, 1),
            "tail_frac": round((span - full_until) / span, 4)}


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1000000,983040,1966080").split(",")]
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    ver = gvm.Verifier([0])
    L = ver._L
    L.gv_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    res = {"lib": os.environ["GV_LIB"], "runs": []}
    for n in sizes:
        pub, sig, dig, exp = bench.make_digest_workload(n, 0xC2, 65536, 0.0, 16)
        d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
        d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
        for p, a in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, a)
        ver.set_option("time_kernels", 1)
        for rep in range(4):                  # back-to-back launches: the clock settles
            ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
        ver.dev_sync()
        ver.stage_stats4()
        ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
        ver.dev_sync()
        cnt, ms = ver.stage_stats4()
        nw = (n + 63) // 64
        buf = np.zeros(2 * 65536 * 6, np.uint64)
        assert L.gv_diag_stamps(ver._ctx, 0, buf.ctypes.data, buf.size) == 0
        st = buf[65536 * 6:].reshape(65536, 6)[:nw].astype(np.int64)
        a = analyse(st, nw)
        a.update({"n": n, "ecmult_ms_event": round(ms[3], 4), "prep_ms_event": round(ms[2], 4)})
        res["runs"].append(a)
        print(json.dumps(a), flush=True)
        for p in d + [d_bits]:
            ver.dev_free(p)
    ver.close()
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
