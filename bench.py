#!/usr/bin/env python3
"""bench.py -- secp256k1 verifies/s on MI355X (BASELINE.json "metric").

Workload (BASELINE.json configs[1]): per rank, 1,000,000
random secp256k1 signatures over 32-byte SHA-256 digests, 65,536 distinct keys
used round-robin, low-S ECDSA signatures (made with OpenSSL by
tools/workload/libgvwork.so; keys per tendermint GenPrivKeySecp256k1).
One "step" = one pass of the hot path (k_unpack -> k_prep -> k_ecmult through
gv_dev_verify_digests) over the whole resident batch.  Inputs are already in
HBM when the timed region starts; the packed accept bitmap stays on device.

Multi-GPU: one process per GPU (torch.distributed.run); each rank verifies its
own independent shard -- no data-path collective.  gloo is used
only for the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line (rank 0).  Extra fields: roofline (integer-VALU bound,
peak = measured v_mad_u64_u32 rate), cpu_baseline (the oracle C port timed on
this host's cores), CheckTx small-batch latency (host path, PCIe included),
and the bitmap parity check of the timed batch against the known verdicts.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "cosmos-sdk-rootchain_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)

import gpuverify as gvm  # noqa: E402

# Work per verify W, in 32x32->64-bit multiply products of
# the 8 x 32 layout (field mul = 64 + 8 = 72, field square = 36 + 8 = 44,
# mod-n Montgomery product = 136), counted from each kernel's own operations
# and attributed to the kernel that does them:
FM, FS, NM = 72, 44, 136
# field operations of the kernels' group law (csrc/secp_group29x.cuh,
# secp_group29.cuh): Jacobian doubling 3M + 4S; mixed addition of a table
# entry scaled by az (gej29x_add_scaled) 8M + 3S; a G entry's lift az = Z zq
# 1M; a lambda-Q entry's beta x 1M; final check (ecmult_finish) Z zq, its
# square and r Z^2: 2M + 1S.  The first addition of a ladder takes the entry
# (no products); a zero digit skips its addition.
DBL, MADD, LIFT, BETA, FINISH = 3 * FM + 4 * FS, 8 * FM + 3 * FS, FM, FM, 2 * FM + FS


def w_ladder(ndbl: int, nq: int, ng: int, qw: int, nbeta: float | None = None, gframe: bool = False) -> float:
    """Expected products of one ladder: ndbl doublings, nq Q-type additions (half
    of them lambda-Q; a qw-bit Booth digit is zero with probability 2 /
    2^(qw+1)), ng lifted G additions, the final check.  Beta products: one per
    lambda-Q addition, or nbeta (the k4 ladders' lambda frame, GV_LAMFRAME:
    two per ladder position).  gframe (k_ecmult_kn, GV_KN_GFRAME, round 6): the
    accumulator moves onto the real curve once before the G additions (1M), so
    they take no lift and the final check no Z zq product."""
    q = nq * (1 - 2.0 / 2 ** (qw + 1))
    nb = q / 2 if nbeta is None else nbeta
    if gframe:
        return ndbl * DBL + (q - 1) * MADD + nb * BETA + FM + ng * MADD + FINISH - FM
    return ndbl * DBL + (q - 1) * MADD + nb * BETA + ng * (MADD + LIFT) + FINISH


W_DECOMP = 255 * FS + 15 * FM              # ParsePubKey: x^3 + 7, the (p+1)/4 chain, y^2 check   12,300
# per-item Q table (build_q_table): co-Z doubling 1M + 5S, 14 co-Z additions
# 5M + 2S, back-propagation 15 x (3M + 1S) + 13 ratio products, Z 1M
W_QTAB = (1 + 14 * 5 + 15 * 3 + 13 + 1) * FM + (5 + 14 * 2 + 15) * FS
W_LADDER = w_ladder(125, 52, 14, 5)        # per-item k_ecmult: 125 doublings, 5-bit Q, 20-bit G windows
W_LADDER_F = w_ladder(125, 52, 11, 5)      # per-item k_ecmult<false, true> ("gfull_item"): G on the unsplit u1
# k_scalar_inv: per item to_mont + the running product (forward), 2 products
# (backward); per lane (GV_INV_M = 32 items) the wave scans (12 + 2
# products), the Montgomery <-> plain conversions of the wave total (3) and
# the shared inversion by variable-time divsteps (secp_modinv.cuh
# s30_modinv_var: ~13 rounds of 30 divsteps for a random 256-bit input, each
# round's matrix applied to (f, g) and (d, e): 4 x 9 + 4 x 9 + 2 x 9
# products), which every lane executes.  (Rounds 1-4 charged the Fermat
# chain's ~340 products here; the kernel has run divsteps since round 3.)
W_DIVSTEPS = 13 * (36 + 36 + 18)
W_INV = 4 * NM + ((14 + 3) * NM + W_DIVSTEPS) / 32
# k_prep's scalar work: u1 = e w, u2 = r w (2 Montgomery products) and two
# GLV splits (2 x 256x256 rounding products + 68 for c1 B1, c2 A1, c1 A1, c2 A2)
W_SCALAR = 2 * NM + 2 * (2 * 64 + 68)
W_KERNEL = {"k_scalar_inv": W_INV,
            "k_prep": W_DECOMP + W_QTAB + W_SCALAR,
            "k_ecmult": W_LADDER}
W_MUL = sum(W_KERNEL.values())
# In-batch key grouping (gv_set_option "group_keys", the default for pub33
# batches with few distinct keys): each distinct key's tables are built once
# (k_keys_chain: ParsePubKey + the doublings to the last group offset;
# k_keys_tables, per group of NT entries: co-Z doubling 1M + 5S, NT - 2 co-Z
# additions with the running Z product 6M + 2S, rho and the last entry
# 6M + 1S, back-propagation (NT - 1)(3M + 1S) + (NT - 2) ratio products; the
# three parked group Zs 1M each) and the items run the keyed pipeline.


def w_keybuild(nt: int, last_offset: int, ng: int = 4) -> float:
    # per group: rho over the other ng - 1 groups' E and the common Z (ng - 1 products; 3 for the quad)
    grp = (1 + (nt - 2) * 6 + (ng + 2) + (nt - 1) * 3 + (nt - 2)) * FM + (5 + (nt - 2) * 2 + 1 + (nt - 1)) * FS
    return W_DECOMP + last_offset * DBL + ng * grp + (ng - 1) * FM


W_KEYBUILD_K4 = w_keybuild(16, 100)        # 4 groups of 16 entries, offsets 0/35/70/100
W_KEYBUILD_K6 = w_keybuild(32, 102)        # 4 groups of 32 entries, offsets 0/36/72/102


def kg_layout(ng: int) -> tuple[int, int]:
    """(ladder positions P, last group's bit offset) of the kg layout KLayout<5, ng>
    (gv_kernels.hip): 26 five-bit windows, the first R groups with P windows."""
    p = -(-26 // ng)
    r = 26 - (p - 1) * ng
    k = ng - 1
    return p, 5 * (k * p - (k - r if k > r else 0))


def w_keybuild_kg(ng: int) -> float:
    return w_keybuild(16, kg_layout(ng)[1], ng)


def w_ladder_kg(ng: int) -> float:
    """k_ecmult_kn<5, ng>: 5 (P - 1) doublings, 52 Q additions (2 beta products per position), 11 G
    additions after the last doubling on the real curve"""
    p = kg_layout(ng)[0]
    return w_ladder(5 * (p - 1), 52, 11, 5, nbeta=2 * p, gframe=True)
W_PREP_KEYED = W_SCALAR
W_PREP_KEYED_F = 2 * NM + (2 * 64 + 68)   # k4f: u2's GLV split only (u1 is recoded unsplit)
# k_ecmult_k4: 30 doublings, 52 Q (26 lambda, on the lambda frame: 2 beta products at each of 7 positions), 14 G additions
W_LADDER_K4 = w_ladder(30, 52, 14, 5, nbeta=14)
# k_ecmult_k6: 30 doublings, 44 Q (22 lambda, on the lambda frame: 2 beta products at each of 6 positions),
# 11 G additions (G on the unsplit u1, 24-bit windows)
W_LADDER_K6 = w_ladder(30, 44, 11, 6, nbeta=12, gframe=True)
# k_ecmult_kn<11> (the resident arena's k6 tables, option keys_k6): 11 groups of two 6-bit windows, 2 positions:
# 6 doublings, 44 Q (22 lambda, 2 beta products per position), 11 G additions
W_LADDER_KN = w_ladder(6, 44, 11, 6, nbeta=4, gframe=True)
# k_ecmult_kn<qw, ceil(130 / qw)> (the resident arena's wide-window tables, option keys_wide 2; qw = the
# library's gv_get_option("kw_qw"), 11 by default): one qw-bit window per group, one position: no doublings,
# 2 ceil(130 / qw) Q (half lambda, 2 beta products), 11 G additions.  keys_wide 1 (or an arena past the
# one-window layout's room): two windows per group, 2 positions: qw doublings, 4 beta products.
def w_ladder_kw(qw: int = 11, two_windows: bool = False) -> float:
    nq = 2 * ((130 + qw - 1) // qw)
    return w_ladder(qw if two_windows else 0, nq, 11, qw, nbeta=4 if two_windows else 2, gframe=True)


W_LADDER_KW = w_ladder_kw(11)
W_LADDER_KW2 = w_ladder_kw(11, True)
W_LADDER_K4F = w_ladder(30, 52, 11, 5, nbeta=14)   # k_ecmult_k4<true>: G on the unsplit u1, 11 25-bit windows
# Peak: the highest v_mad_u64_u32 issue rate measured on MI355X
# (tools/microbench/alu_rate.hip; profiles/r01/alu_rate_v3.jsonl, dependent
# chains at 8 waves/SIMD), lane-products per second, whole chip.  bench.py
# also re-measures it live and uses the larger of the two.
P_MUL_COMMITTED = 3.7469e13
ALU_BENCH = os.path.join(REPO, "tools", "microbench", "alu_rate")

WORKLOAD_SO = os.path.join(REPO, "tools", "workload", "libgvwork.so")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload_lib():
    if not os.path.exists(WORKLOAD_SO):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.dirname(WORKLOAD_SO)], check=True)
    L = ctypes.CDLL(WORKLOAD_SO)
    L.gvw_keys.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.gvw_sign.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.gvw_openssl_verify.argtypes = [ctypes.c_size_t] + [ctypes.c_void_p] * 7 + [ctypes.c_int]
    return L


def make_digest_workload(n: int, seed: int, nkeys: int, adv: float, threads: int):
    L = workload_lib()
    priv = np.zeros((nkeys, 32), np.uint8)
    pubk = np.zeros((nkeys, 33), np.uint8)
    L.gvw_keys(nkeys, seed, priv.ctypes.data, pubk.ctypes.data, threads)
    pub = np.zeros((n, 33), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    dig = np.zeros((n, 32), np.uint8)
    exp = np.zeros(n, np.uint8)
    L.gvw_sign(n, seed, nkeys, priv.ctypes.data, pubk.ctypes.data, None, None, adv, pub.ctypes.data,
               sig.ctypes.data, dig.ctypes.data, exp.ctypes.data, threads)
    return pub, sig, dig, exp


def unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]


def openssl_verify(pub, sig, dig=None, msgs=None, threads: int = 1):
    """tools/workload gvw_openssl_verify: VerifyBytes semantics on OpenSSL."""
    L = workload_lib()
    n = len(pub)
    out = np.zeros(n, np.uint8)
    if dig is not None:
        L.gvw_openssl_verify(n, pub.ctypes.data, sig.ctypes.data, dig.ctypes.data, None, None, None,
                             out.ctypes.data, threads)
    else:
        blob, off, ln = msgs
        L.gvw_openssl_verify(n, pub.ctypes.data, sig.ctypes.data, None, blob.ctypes.data, off.ctypes.data,
                             ln.ctypes.data, out.ctypes.data, threads)
    return out


def _rate(fn, n):
    t = time.perf_counter()
    fn()
    return round(n / (time.perf_counter() - t), 1)


def cpu_baseline(pub, sig, dig, threads: int, ver=None):
    """CPU timing beside the GPU: (ii) the oracle port
    (oracle/secp256k1_oracle.c, the reference algorithm restated in C) and
    (iii) OpenSSL (ECDSA_do_verify + the low-S rule), each serial and on
    `threads` cores, on bounded samples of C2 (digests) and of the C1 item set
    (10k MsgSend StdSignBytes messages: SHA-256 + verify).  (i), the Go
    reference, needs a Go toolchain the box does not have.  `value` is the
    oracle port on C2, all cores.  The C1 line also times the GPU host path
    (gv_verify_msgs, PCIe included) on the same 10k items."""
    from oracle import oracle as O
    O.lib()
    s1 = 4096
    # all-core sample sized for ~6 s from a short calibration run
    cal = min(len(pub), 512 * threads)
    t = time.perf_counter()
    O.verify_digests(pub[:cal], sig[:cal], dig[:cal], threads=threads)
    est = cal / (time.perf_counter() - t)
    s2 = int(min(len(pub), max(cal, est * 6)))
    c2 = {
        "port_serial": _rate(lambda: O.verify_digests(pub[:s1], sig[:s1], dig[:s1], threads=1), s1),
        "port_allcore": _rate(lambda: O.verify_digests(pub[:s2], sig[:s2], dig[:s2], threads=threads), s2),
        "openssl_serial": _rate(lambda: openssl_verify(pub[:s1], sig[:s1], dig[:s1], threads=1), s1),
        "openssl_allcore": _rate(lambda: openssl_verify(pub[:s2], sig[:s2], dig[:s2], threads=threads), s2),
    }
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_extras as X
    n1 = 10000
    cpub, csig, cmsgs, cexp = X.c1_items(workload_lib(), n1, threads)
    blob, off, ln = cmsgs
    c1 = {
        "items": n1, "mean_msg_bytes": round(float(ln.mean()), 1),
        "port_serial": _rate(lambda: O.verify_msgs(cpub[:s1], csig[:s1], blob, off[:s1], ln[:s1], threads=1), s1),
        "port_allcore": _rate(lambda: O.verify_msgs(cpub, csig, blob, off, ln, threads=threads), n1),
        "openssl_serial": _rate(lambda: openssl_verify(cpub[:s1], csig[:s1], msgs=(blob, off[:s1], ln[:s1]),
                                                       threads=1), s1),
        "openssl_allcore": _rate(lambda: openssl_verify(cpub, csig, msgs=cmsgs, threads=threads), n1),
    }
    if ver is not None:
        ver.verify_batch_msgs(cpub, csig, cmsgs)                # warm the message-path buffers
        t = time.perf_counter()
        got = ver.verify_batch_msgs(cpub, csig, cmsgs)
        c1["gpu_hostpath"] = round(n1 / (time.perf_counter() - t), 1)
        c1["gpu_mismatches"] = int(np.count_nonzero(got != cexp))
    return {"value": c2["port_allcore"], "unit": "verifies/s", "cores": threads, "kind": "port",
            "label": "no-GLV C restatement, not btcec (the reference's btcec uses GLV and would likely be faster; "
                     "the Go toolchain is absent, so the reference itself cannot be timed): a reported baseline, "
                     "never a target",
            "host": host_cores(),
            "sample": f"first {s2} items of the same C2 batch, {threads} threads = every CPU this process may run on "
                      f"(affinity mask, capped by the cgroup quota; see host) (oracle/secp256k1_oracle.c: a clarity-first 4x64-limb port of the reference "
                      f"algorithm, no GLV); serial 1-thread on the first {s1}; OpenSSL and the C1 message set "
                      f"beside it (SURVEY.md §8d lines ii and iii)",
            "serial_value": c2["port_serial"], "c2": c2, "c1": c1}


def live_mad_peak():
    """Max v_mad_u64_u32 lane-products/s measured now by tools/microbench/alu_rate (None if unavailable)."""
    import subprocess
    if not os.path.exists(ALU_BENCH):
        return None
    try:
        out = subprocess.run([ALU_BENCH], capture_output=True, text=True, timeout=120).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    best = None
    for line in out.splitlines():
        try:
            d = json.loads(line)
        except ValueError:
            continue
        if str(d.get("inst", "")).startswith("v_mad_u64_u32"):
            best = max(best or 0.0, float(d["lane_ops_per_s"]))
    return best


def host_cores():
    """CPU counts of this host: os.cpu_count(), the affinity mask, and the cgroup
    CPU quota (cpu.max) when one is set."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    eff = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "effective": eff}


def _pct(ts):
    ts = np.array(ts) * 1e3
    return round(float(np.percentile(ts, 50)), 3), round(float(np.percentile(ts, 99)), 3)


def checktx_latency(ver, pub, sig, dig, threads, sizes=(1, 16, 32, 64, 128, 256, 1024, 4096), reps=1000):
    """C5: host-path latency (host buffers in -> verdicts out) per batch size.
    p50/p99 are the default GPU path: up to "lat_sl_max" (2048) the limb-sliced
    small-batch kernels (gv_lat.hip k_verify_lat_sl4 up to "lat_rows_max" = 512,
    k_verify_lat_sl above / k_verify_lat16_sl keyed, one signature per block)
    reading the pinned staging buffer zero-copy, up to
    "lat_max" (8192) the four-lanes-per-signature kernel, the pipeline above
    ("schedule" per size); next to it the throughput pipeline forced for the
    same batches, the message path (gv_verify_msgs over ~355-byte StdSignBytes:
    SHA-256 on the GPU, "msgs_p50_ms"), the keyed path (account keys in the HBM key arena,
    gv_verify_digests_keyed), and the CPU oracle (oracle/secp256k1_oracle.c,
    the reference algorithm restated in C) serial and on `threads` cores."""
    from oracle import oracle as O
    if os.path.join(REPO, "tools") not in sys.path:
        sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_extras as X
    O.lib()
    out = {}
    # the message path (gv_verify_msgs: SHA-256 of the StdSignBytes on the GPU,
    # what the Go drop-in's CheckTx calls): 4,096 C1 sign-bytes items
    mn = 4096
    mpub, msig, (mblob, moff, mln), _ = X.c1_items(workload_lib(), mn, threads, 1024)
    nkeys = 65536                                   # the C2 workload's keys, item i uses key i % nkeys
    ver.keys_reset()
    slots = ver.keys_load(pub[:nkeys])[np.arange(len(pub)) % nkeys]
    for b in sizes:
        def run_gpu(rr):
            ts = []
            for r in range(rr + 5):
                o = (r * b) % (len(pub) - b)
                t = time.perf_counter()
                ver.verify_batch_digests(pub[o:o + b], sig[o:o + b], dig[o:o + b])
                ts.append(time.perf_counter() - t)
            return ts[5:]
        p50, p99 = _pct(run_gpu(reps))
        ts = []
        for r in range(reps // 2 + 5):
            o = (r * b) % (len(pub) - b)
            t = time.perf_counter()
            ver.verify_batch_digests_keyed(slots[o:o + b], sig[o:o + b], dig[o:o + b])
            ts.append(time.perf_counter() - t)
        keyed50, _ = _pct(ts[5:])
        ts = []
        for r in range(reps // 2 + 5):
            o = (r * b) % (mn - b) if b < mn else 0
            t = time.perf_counter()
            ver.verify_batch_msgs(mpub[o:o + b], msig[o:o + b], (mblob, moff[o:o + b], mln[o:o + b]))
            ts.append(time.perf_counter() - t)
        msgs50, _ = _pct(ts[5:])
        ver.set_option("lat_max", 0)
        tp50, _ = _pct(run_gpu(max(20, reps // 4)))
        ver.reset_schedule()
        cpu = {}
        for label, th in (("cpu_serial_p50_ms", 1), ("cpu_allcore_p50_ms", threads)):
            ts = []
            budget = time.perf_counter() + 1.0
            for r in range(50):
                o = (r * b) % (len(pub) - b)
                t = time.perf_counter()
                O.verify_digests(pub[o:o + b], sig[o:o + b], dig[o:o + b], threads=th)
                ts.append(time.perf_counter() - t)
                if time.perf_counter() > budget and len(ts) >= 3:
                    break
            cpu[label] = _pct(ts)[0]
        sched = ("k_verify_lat_sl4 (limb-sliced, row-parallel ladders, zero-copy)" if b <= gvm.LAT_ROWS_MAX_DEFAULT else
                 "k_verify_lat_sl (limb-sliced, zero-copy)" if b <= gvm.LAT_SL_MAX_DEFAULT else
                 "k_verify_lat (4 lanes per signature)" if b <= gvm.LAT_MAX_DEFAULT else "pipeline")
        out[str(b)] = {"p50_ms": p50, "p99_ms": p99, "throughput_path_p50_ms": tp50, "keyed_p50_ms": keyed50,
                       "msgs_p50_ms": msgs50, **cpu, "schedule": sched}
    ver.keys_reset()
    return out


PMC_SUMMARY = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_latest.json")


def load_pmc(kernel):
    """Per-item HBM bytes / VALU counters of `kernel` from the committed PMC summary
    (tools/pmc_summary.py over tools/pmc_round.sh); None if absent."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        e = dict(d["kernels"][kernel])
        e["source"] = d["source"]
        return e
    except (OSError, KeyError, ValueError):
        return None


def main(argv=None, verifier_factory=None, workload_fn=None):
    """verifier_factory(local_rank) / workload_fn(n, seed, keys, adv, threads) are
    injection points for tests/test_bench_dist.py (gloo, CPU, fake verifier)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--items", "--n", dest="n", type=int, default=1_000_000, help="signatures per rank")
    ap.add_argument("--adversarial", type=float, default=0.0, help="C3: fraction of invalid signatures")
    ap.add_argument("--keys", type=int, default=65536)
    ap.add_argument("--threads", type=int, default=host_cores()["effective"] or 1,
                    help="CPU baseline / workload threads (default: every CPU this process may run on: the "
                         "affinity mask, capped by the cgroup CPU quota when one is set)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the C3 / message-path / C1 / C4 lines")
    ap.add_argument("--inproc", action="store_true",
                    help="the node's shape: ONE process, one gv_open over --gpus devices (0 = every visible one), "
                         "gv_verify_digests_bits from host buffers of items x devices signatures; per-device rates")
    args = ap.parse_args(argv)
    if args.inproc:
        return run_inproc(args, verifier_factory, workload_fn)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    n = args.n
    t0 = time.perf_counter()
    pub, sig, dig, exp = (workload_fn or make_digest_workload)(n, 0xC2 + 7919 * rank, args.keys, args.adversarial,
                                                               args.threads)
    log(f"[rank {rank}] workload {n} items in {time.perf_counter() - t0:.1f}s; valid {exp.mean():.3f}")

    ver = verifier_factory(local_rank) if verifier_factory else gvm.Verifier([local_rank])
    d_pub = ver.dev_alloc(pub.nbytes)
    d_sig = ver.dev_alloc(sig.nbytes)
    d_dig = ver.dev_alloc(dig.nbytes)
    nwords = (n + 63) // 64
    d_bits = ver.dev_alloc(nwords * 8)
    ver.dev_upload(d_pub, pub)
    ver.dev_upload(d_sig, sig)
    ver.dev_upload(d_dig, dig)

    def step():
        ver.dev_verify_digests(0, n, d_pub, d_sig, d_dig, d_bits)

    for _ in range(args.warmup):
        step()
    ver.dev_sync()

    # parity of the resident batch against the verdicts known by construction
    bits = np.zeros(nwords, np.uint64)
    ver.dev_download(bits, d_bits)
    got = unpack_bits(bits, n)
    mismatches = int(np.count_nonzero(got != exp))

    # parity on an adversarial copy of the same batch (a kernel that accepted
    # everything would pass the all-valid check above): 1/8 of the items get a
    # malformed pubkey prefix (ParsePubKey rejects), 1/8 a flipped digest bit
    # (ECDSA rejects); expected verdicts by construction
    rng = np.random.default_rng(0xADF + rank)
    sel = rng.random(n)
    bad_pfx, bad_dig = sel < 0.125, (sel >= 0.125) & (sel < 0.25)
    apub, adig = pub.copy(), dig.copy()
    apub[bad_pfx, 0] = 0x05
    adig[bad_dig, 31] ^= 1
    aexp = exp & ~(bad_pfx | bad_dig)
    ver.dev_upload(d_pub, apub)
    ver.dev_upload(d_dig, adig)
    step()
    ver.dev_sync()
    ver.dev_download(bits, d_bits)
    adv_mismatches = int(np.count_nonzero(unpack_bits(bits, n) != aexp))
    adv_rejected = int(n - aexp.sum())
    ver.dev_upload(d_pub, pub)
    ver.dev_upload(d_dig, dig)
    del apub, adig

    ver.set_option("time_kernels", 1)
    ver.stage_stats4()                    # reset the event ring
    barrier()
    ver.dev_sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    ver.dev_sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    cnt_p, pipe_stages = ver.stage_stats4()
    grp0 = ver.group_stats() if hasattr(ver, "group_stats") else (0, 0)
    routes0 = ver.route_stats() if hasattr(ver, "route_stats") else {}
    # The timed loop is pipelined (gv_set_option "pipeline_dev": call k+1's
    # front kernels run under call k's ladder), so its kernels overlap and
    # their event durations include each other.  Each kernel's own speed --
    # the roofline's denominator -- comes from a serialized calibration pass
    # of the same batch right after the timed loop (the last `calib` launches
    # of every kernel: tools/prof_timed.py picks the same ones from a trace).
    calib = args.steps
    ver.set_option("pipeline_dev", 0)
    for _ in range(calib):
        step()
    ver.dev_sync()
    cnt, (unpack_ms, inv_ms, prep_ms, ecmult_ms) = ver.stage_stats4()
    ver.set_option("pipeline_dev", 1)
    ver.set_option("time_kernels", 0)
    elapsed_max = allmax(elapsed)
    total_mismatch = int(allmax(float(mismatches)))
    total_adv_mismatch = int(allmax(float(adv_mismatches)))

    value = world * n * args.steps / elapsed_max
    ms_per_step = elapsed_max / args.steps * 1e3

    peak_live = live_mad_peak() if rank == 0 else None
    P_MUL = max(P_MUL_COMMITTED, peak_live or 0.0)
    # which pipeline the calibration launches took: in-batch key grouping
    # (the keyed route) or the per-item pub33 route
    gb, gk = (ver.group_stats() if hasattr(ver, "group_stats") else (0, 0))
    grouped = gb - grp0[0] >= calib
    u_keys = (gk - grp0[1]) / max(1, gb - grp0[0]) if grouped else 0.0
    routes1 = ver.route_stats() if hasattr(ver, "route_stats") else {}
    k6 = grouped and routes1.get("k6", 0) - routes0.get("k6", 0) >= calib
    kg = ver.get_option("kg") if grouped and routes1.get("kg", 0) - routes0.get("kg", 0) >= calib else 0
    k4f = grouped and routes1.get("k4f", 0) - routes0.get("k4f", 0) >= calib
    itemf = not grouped and routes1.get("item_f", 0) - routes0.get("item_f", 0) >= calib
    if grouped:
        # the key tables (k_keys_chain, k_keys_tables) run on a side stream
        # beside k_scalar_inv: that stage's time covers both
        lad = f"k_ecmult_kn<5, {kg}>" if kg else "k_ecmult_k6" if k6 else "k_ecmult_k4"
        wkb = w_keybuild_kg(kg) if kg else W_KEYBUILD_K6 if k6 else W_KEYBUILD_K4
        w = {"k_unpack+k_dedupe": 0.0, "k_scalar_inv|k_keys_chain+k_keys_tables": W_INV + wkb * u_keys / n,
             "k_prep<keyed>": W_PREP_KEYED_F if (k4f or k6 or kg) else W_PREP_KEYED,
             lad: w_ladder_kg(kg) if kg else W_LADDER_K6 if k6 else W_LADDER_K4F if k4f else W_LADDER_K4}
        kms = dict(zip(w, (unpack_ms, inv_ms, prep_ms, ecmult_ms)))
        ladder, w_route = lad, sum(w.values())
    else:
        w = dict(W_KERNEL)
        if itemf:                                  # one GLV split fewer in k_prep, 11 G additions
            w["k_prep"] = W_DECOMP + W_QTAB + 2 * NM + (2 * 64 + 68)
            w["k_ecmult"] = W_LADDER_F
        kms = {"k_scalar_inv": inv_ms, "k_prep": prep_ms, "k_ecmult": ecmult_ms}
        ladder, w_route = "k_ecmult", sum(w.values())
    kernels = {}
    for k, ms in kms.items():
        a = n * w[k] / (ms * 1e-3) if ms > 0 else 0.0
        kernels[k] = {"ms": round(ms, 4), "work_per_verify": round(w[k]), "achieved_T": round(a / 1e12, 3),
                      "frac": round(a / P_MUL, 4) if a else None}
    achieved = n * w[ladder] / (ecmult_ms * 1e-3) if ecmult_ms > 0 else 0.0
    pmc = load_pmc(ladder)
    traffic = round(pmc["hbm_bytes_per_item"] * n) if pmc else None
    result = {
        "metric": "secp256k1 verifies/sec at 1/2/4/8 MI355X; p50 latency @64-tx CheckTx batch",
        "value": round(value, 1),
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: OpenSSL-signed low-S ECDSA over random SHA-256 digests, 65,536 keys round-robin",
        "config": {"workload": "C2: 1M random secp256k1 sigs over 32-byte sha256 digests per GPU "
                               "(bit-exact bitmap vs btcec semantics)",
                   "items_per_gpu": n, "keys": args.keys, "adversarial_fraction": args.adversarial,
                   "global_batch": n * world, "parallelism": f"shard{world} (independent per-GPU shards, no collective)",
                   "route": ("in-batch key grouping: each distinct key parsed and tabulated once (k_dedupe, "
                             "k_keys_chain + k_keys_tables), items on the keyed "
                             + (f"{5 * (kg_layout(kg)[0] - 1)}-doubling ladder k_ecmult_kn<5, {kg}> ({kg} groups of "
                                "16-entry 5-bit tables, G after the last doubling from 11 24-bit windows on the real "
                                "curve)" if kg else "30-doubling ladder ")
                             + ("" if kg else "k_ecmult_k6 (6-bit Q windows on 32-entry key tables, G on the unsplit "
                                "scalar: 11 24-bit windows)" if k6
                                else "k_ecmult_k4 (G on the unsplit scalar: 11 25-bit windows)" if k4f
                                else "k_ecmult_k4 (GLV G: 14 20-bit windows)")
                             if grouped else "per-item pub33 pipeline (every item decompresses its key)"),
                   "distinct_keys_per_batch": round(u_keys) if grouped else None},
        "roofline": {
            "bound": "valu",
            "kernel": ladder,
            "achieved": round(achieved / 1e12, 3),
            "peak": round(P_MUL / 1e12, 3),
            "unit": "Tmul32/s",
            "frac": round(achieved / P_MUL, 4) if achieved else None,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE, scaled per item)",
            "traffic_source": pmc["source"] if pmc else None,
            "hbm_gbps_at_traffic": round(traffic / (ecmult_ms * 1e-3) / 1e9, 1) if (pmc and ecmult_ms > 0) else None,
            "valu_insts_per_verify": round(pmc["valu_insts_per_item"]) if pmc else None,
            "valu_busy_frac": round(pmc["valu_busy_frac"], 3) if pmc else None,
            "work_per_verify": round(w[ladder]),
            "kernel_ms": round(ecmult_ms, 4),
            "launches_averaged": cnt,
            "kernel_ms_source": "serialized calibration pass after the timed loop (the ladder's own launch "
                                "duration, HIP events); in the pipelined timed loop the kernels overlap",
            "peak_committed": round(P_MUL_COMMITTED / 1e12, 3),
            "peak_live": round(peak_live / 1e12, 3) if peak_live else None,
            "kernels": kernels,
            "note": "achieved = items x W (32x32 products per verify, SURVEY §8d, attributed per kernel: the Q-table "
                    "build belongs to k_prep) / avg kernel duration (HIP events on the launch stream); peak = the "
                    "max of the committed and live-measured v_mad_u64_u32 chip rates; traffic / VALU counters from "
                    "the committed rocprofv3 --pmc passes of this bench command (tools/pmc_round.sh)",
        },
        "pipeline": {"unpack_ms": round(unpack_ms, 3), "scalar_inv_ms": round(inv_ms, 3),
                     "prep_ms": round(prep_ms, 3), "ecmult_ms": round(ecmult_ms, 3),
                     "serialized_sum_ms": round(unpack_ms + inv_ms + prep_ms + ecmult_ms, 3),
                     "pipelined_ms_per_step": round(ms_per_step, 3),
                     "pipelined_overlapped_stage_ms": [round(x, 3) for x in pipe_stages],
                     "pipelined_launches": cnt_p,
                     "whole_verify_work_per_verify": round(w_route),
                     "whole_verify_roofline_frac": round(value / world * w_route / P_MUL, 4),
                     "note": "timed steps are pipelined: call k+1's unpack / s^-1 / prep run on a low-priority "
                             "stream under call k's ladder (high-priority stream); stage ms above from the "
                             "serialized calibration pass, the overlapped ones beside them"},
        "parity": {"checked": n * world, "mismatches": total_mismatch,
                   "adversarial_checked": n * world, "adversarial_rejects_expected": adv_rejected * world,
                   "adversarial_mismatches": total_adv_mismatch,
                   "reference": "verdicts known by construction: the timed batch (valid signatures) and an "
                                "adversarial copy (1/8 malformed prefix, 1/8 flipped digest bit -> rejected)"},
    }

    lat = None
    if rank == 0 and world == 1 and not args.no_latency:
        lat = checktx_latency(ver, pub, sig, dig, args.threads)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(pub, sig, dig, args.threads, ver)
        result["cpu_baseline"] = cb
        result["gpu_over_cpu"] = round(value / cb["value"], 1)
        result["gpu_over_openssl_allcore"] = round(value / cb["c2"]["openssl_allcore"], 1)

    for p in (d_pub, d_sig, d_dig, d_bits):
        ver.dev_free(p)
    if rank == 0 and world == 1 and not args.no_extras:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import bench_extras as X
        ex = {}
        t = time.perf_counter()
        ex["c2_hostpath"] = X.c2_hostpath(ver, pub, sig, dig, exp, device_value=value)
        ex["c2_key_cache"] = X.c2_key_cache(ver, pub, sig, dig, exp, min(args.keys, n))
        ex["c2_unique_keys"] = X.c2_unique_keys(ver, make_digest_workload, n, args.threads)
        ex["c2_per_item_parse"] = X.c2_per_item_parse(ver, pub, sig, dig, exp)
        ex["c3_adversarial"] = X.c3_adversarial(ver, make_digest_workload, n, args.threads)
        ex["msg_path"] = X.msg_path(ver, workload_lib(), min(n, 500_000), args.threads)
        ex["c1_ante"] = X.c1_ante(ver, wl=workload_lib(), threads=min(args.threads, 16))
        ex["c4_multisig"] = X.c4_multisig(ver, workload_lib(), threads=min(args.threads, 16))
        ex["ed25519"] = X.ed25519(ver, workload_lib(), n=n, threads=args.threads, peak=P_MUL)
        # last: tearing down first_call's second context (12 GiB of G tables
        # freed) slows the next few host-path calls of this one by ~20 %
        # (tools/hostpath_probe.py: bits_pinned 6.28 -> 7.75 ms right after it)
        ex["first_call"] = X.first_call(pub, sig, dig, exp)
        log(f"extras in {time.perf_counter() - t:.1f}s")
        result["extras"] = ex
        result["summary"] = summarize(result, ex)
    if lat is not None:
        # BASELINE's second number, last in the line so that a truncated tail
        # of stdout still shows it: the full curve, then p50 @ 64
        result["checktx_latency_ms"] = lat
        result["checktx_p50_ms_64"] = lat["64"]["p50_ms"]
    ver.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def summarize(result, ex):
    """One compact block of the side lines, placed right before the C5 curve
    at the end of the JSON line so that a truncated tail of stdout still
    carries them: the node paths (host buffers, C1, C4), the other C2 routes
    and their rooflines from serialized passes, ed25519."""
    def g(d, *path):
        for k in path:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d
    v = result["value"]
    return {
        "c2_device_resident": v,
        "c2_hostpath": {"pageable": g(ex, "c2_hostpath", "value"), "pinned": g(ex, "c2_hostpath", "value_pinned"),
                        "frac_pageable": g(ex, "c2_hostpath", "frac_of_device_resident"),
                        "frac_pinned": g(ex, "c2_hostpath", "frac_of_device_resident_pinned"),
                        "async": g(ex, "c2_hostpath", "value_async"),
                        "async_pinned": g(ex, "c2_hostpath", "value_async_pinned"),
                        "frac_async": g(ex, "c2_hostpath", "frac_of_device_resident_async"),
                        "frac_async_pinned": g(ex, "c2_hostpath", "frac_of_device_resident_async_pinned")},
        "c2_key_cache": {"value": g(ex, "c2_key_cache", "value"), "route": g(ex, "c2_key_cache", "route"),
                         "frac": g(ex, "c2_key_cache", "roofline", "frac"),
                         "ladder_ms": g(ex, "c2_key_cache", "roofline", "kernel_ms")},
        "c2_unique_keys": {"value": g(ex, "c2_unique_keys", "value"),
                           "ladder_frac": g(ex, "c2_unique_keys", "roofline", "k_ecmult", "frac"),
                           "front_frac": g(ex, "c2_unique_keys", "roofline", "k_scalar_inv+k_prep", "frac")},
        "c2_per_item_parse": g(ex, "c2_per_item_parse", "value"),
        "c3_adversarial": g(ex, "c3_adversarial", "value"),
        "msg_path": g(ex, "msg_path", "value"),
        "c1_one_block_tx_s": g(ex, "c1_ante", "block_path_steady", "txs_per_s"),
        "c1_replay_tx_s": g(ex, "c1_ante", "replay_pipelined_steady", "txs_per_s"),
        "c4_replay_leaves_s": g(ex, "c4_multisig", "leaves_per_s"),
        "c4_one_block_leaves_s": g(ex, "c4_multisig", "one_block_at_a_time", "leaves_per_s"),
        "ed25519_grouped": g(ex, "ed25519", "value"),
        "ed25519_64_cached_p50_ms": g(ex, "ed25519", "small_batches", "batches", "64", "keyed_sliced_p50_ms"),
        "ed25519_64_uncached_p50_ms": g(ex, "ed25519", "small_batches", "batches", "64", "uncached_p50_ms"),
        "first_call": g(ex, "first_call"),
        "cpu_baseline_kind": "no-GLV C restatement of the reference algorithm (oracle/secp256k1_oracle.c), not btcec: "
                             "the Go reference (btcec with GLV) cannot run here and would likely be faster",
    }


def run_inproc(args, verifier_factory=None, workload_fn=None):
    """SURVEY.md §8e as the Go node runs it: one context over every device
    (gv_open(n_dev=0) in crypto/gpuverify.Open), host buffers in, the library
    splitting the batch into contiguous per-device slices (persistent
    per-device workers, one shared staging pool) and gathering the bitmaps.
    PCIe included (host buffers): this is the node-level rate, not `value` of
    the device-resident line."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--inproc runs as ONE process over all devices (do not launch it with torch.distributed.run)")
    devs = list(range(args.gpus)) if args.gpus > 0 else None
    ver = verifier_factory(devs) if verifier_factory else gvm.Verifier(devs)
    nd = ver.num_devices
    n = args.n * nd
    t0 = time.perf_counter()
    pub, sig, dig, exp = (workload_fn or make_digest_workload)(n, 0xC2, args.keys, args.adversarial, args.threads)
    log(f"[inproc] workload {n} items over {nd} devices in {time.perf_counter() - t0:.1f}s")
    for _ in range(args.warmup):
        bits = ver.verify_batch_digests_bits(pub, sig, dig)
    mismatches = int(np.count_nonzero(unpack_bits(bits, n) != exp))
    t = time.perf_counter()
    for _ in range(args.steps):
        ver.verify_batch_digests_bits(pub, sig, dig)
    elapsed = time.perf_counter() - t
    slices = ver.last_slices()
    ver.close()
    value = n * args.steps / elapsed
    result = {
        "metric": "secp256k1 verifies/sec at 1/2/4/8 MI355X; p50 latency @64-tx CheckTx batch",
        "mode": "inproc",
        "value": round(value, 1), "unit": "verifies/s", "n_gpus": nd, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: OpenSSL-signed low-S ECDSA over random SHA-256 digests, 65,536 keys round-robin",
        "config": {"workload": f"C2 x {nd}: {args.n} signatures per device in ONE host batch (pageable host "
                               f"buffers, PCIe included)", "items_per_gpu": args.n, "global_batch": n,
                   "parallelism": f"inproc{nd} (one gv_ctx over {nd} devices: contiguous slices, "
                                  f"no collective, bitmaps gathered to the host)"},
        "per_device": [{"slot": k, "items": int(c), "slice_ms": round(ms, 3),
                        "verifies_per_s": round(c / (ms * 1e-3), 1) if ms > 0 else None}
                       for k, (ms, c) in enumerate(slices)],
        "parity": {"checked": n, "mismatches": mismatches, "reference": "verdicts known by construction"},
        "host": host_cores(),
    }
    print(json.dumps(result), flush=True)
    return result


if __name__ == "__main__":
    main()
